// wellflow — monotonic hand-off words of the persistent LSTM kernels (lstm_persistent_*.inc.h).
//
// The sync buffer is zeroed ONCE (allocation, NativeLSTM.reset_device_errors) and never by a
// launch: no memset node precedes a persistent launch (round-4 VERDICT item 4; the round-2
// silent early exit was an unaligned per-launch memset node under graph replay,
// profiles/r3_early_exit.md). Every word only counts up:
//   row block m owns words [16 + 16m, 16 + 16m + 16) (one 64-B line):
//     +0        START: each of the row block's NB workgroups adds 1 when it starts, so
//               start_value / NB is the launch's EPOCH for this row block (launches of one
//               buffer are stream-ordered and persistent: all NB adds of launch e precede
//               every add of launch e + 1)
//     +1 .. +8  GROUP g arrivals: each workgroup adds 1 per published row-tile group per step;
//               a consumer's target is epoch * NB * (publishes per launch) + NB * steps, so
//               the counters never need resetting
//     +12       ERROR: the epoch + 1 of the launch in which some workgroup of the row block
//               hit its spin bound (a stale tag from an earlier launch is ignored)
// The 64-word STAT block at the END of the buffer keeps its running totals
// (persistent_guard.h).
// A workgroup that fails a hand-off does NOT return: it marks itself failed, records why, and
// runs to the end without waiting again (results garbage, reported through STAT), so no wave
// can strand another at a barrier or a poll.
#pragma once
#include <hip/hip_runtime.h>

#include "persistent_guard.h"

namespace wf {

constexpr int kPSyncHead = 16;      // words before the first row block (word 0: launch signature)
constexpr int kPSyncRowBlock = 16;  // words per row block
constexpr int kPSyncStart = 0, kPSyncGroup = 1, kPSyncErr = 12;
constexpr int kPSyncMaxGroups = 8;

typedef __attribute__((address_space(1))) unsigned ps_u32;

__device__ __forceinline__ ps_u32* psync_rb(unsigned* sync, int m) {
  return (ps_u32*)(sync + kPSyncHead + kPSyncRowBlock * m);
}

// (counter - target) as a signed distance: the counters may wrap after ~2^31 publishes
__device__ __forceinline__ bool psync_reached(unsigned v, unsigned target) { return (int)(v - target) >= 0; }

// Launch SIGNATURE in head word 0. The epoch targets above assume every launch on one buffer
// published the same number of groups per launch: same kernel, same row tiles per workgroup
// (NC), same steps (T), same column blocks (NB). A launch of another shape on the same buffer
// (e.g. a smaller batch choosing a different NC) would see counters already past its targets
// and read unpublished data (round-5 ADVICE). So the first launch after the buffer is zeroed
// claims word 0 with its signature, and a launch with a different one fails loudly (reason 5,
// every wave runs on without waiting, the STAT check raises) instead of racing.
__device__ __forceinline__ unsigned psync_sig(unsigned kind, unsigned nc, unsigned steps, unsigned nb) {
  return 0x80000000u | ((kind & 3u) << 29) | ((nc & 15u) << 25) | ((nb & 31u) << 20) | (steps & 0xFFFFFu);
}
// thread 0 of every workgroup, before its first wait: 0 = ok, else the conflicting signature
__device__ __forceinline__ unsigned psync_check_sig(unsigned* sync, unsigned sig) {
  unsigned prev = 0u;
  __hip_atomic_compare_exchange_strong((ps_u32*)sync, &prev, sig, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return (prev == 0u || prev == sig) ? 0u : prev;
}

// Blocking wait of ONE wave (every lane runs it, uniform address): relaxed agent-scope (sc1)
// poll of a group counter with s_sleep, bounded; the error word is checked so a failure
// elsewhere in the row block ends the wait. Returns 0 (reached), 1 (another workgroup
// failed) or 2 (own spin bound: sets the error word and the sticky bit).
__device__ __forceinline__ unsigned psync_wait(ps_u32* cnt, ps_u32* err, unsigned target, unsigned tag,
                                               unsigned spin_limit, unsigned* stat, unsigned* seen_cnt,
                                               unsigned* seen_err) {
  unsigned spins = 0;
  while (true) {
    const unsigned v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *seen_cnt = v;
    if (psync_reached(v, target)) return 0;
    const unsigned e = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *seen_err = e;
    if (e == tag) return 1;
    if (++spins > spin_limit) {
      __hip_atomic_store(err, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((threadIdx.x & 63) == 0) pguard_sticky(stat);
      return 2;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

}  // namespace wf
