// wellflow — persistent LSTM backward (BPTT): ONE launch runs steps T-2 .. 0 (kernel template;
// instantiations: lstm_pb_parts.hip, host launcher: lstm_persistent_bwd.hip)
// (SURVEY.md §2.4 K14 "lstm_seq_bwd (persistent)"; the forward twin is lstm_persistent.hip).
//
// Why: the per-step backward (lstm.hip, 63 launches) re-streams its W_hh tile from L2 every
// step (512 KB per 128x128 tile, 134 MB per step over the grid), and round-trips the fp32
// dc carry through HBM (2 x 16.8 MB per step at B = 8192). Here
//  * grid = (B / (16 * NRT)) row blocks x (H / 64) unit blocks, one 256-thread workgroup
//    (4 waves, one per SIMD) per CU, co-resident (persistent_launch.h). Workgroup (m, n)
//    owns rows [16*NRT*m, +16*NRT) x units [64n, 64n + 64) for the whole sequence, i.e.
//    the 256 contiguous DG columns 4u + gate of those units (dg_col order).
//  * dh_t = DG_{t+1} W_hh is split over K by wave: wave w multiplies DG columns
//    [w*H, (w+1)*H) by the matching rows of W_hh, for all 64 units. Its W_hh^T slice
//    (64 units x H k's) stays in AGPRs for the whole sequence (H/2 = 256 registers at
//    H = 512). Its A operand streams through a private 2-slot LDS-DMA ring (buffer_load ...
//    lds, every instruction 8 rows x 128 B: full lines; the pieces of tile r+1 are issued
//    between tile r's MFMAs). The 4 partial 16x64 dh tiles are summed through LDS (deferred
//    into the next tile's loop), each wave then owning one 16-unit tile for the cell backward.
//  * the dc carry of the workgroup's rows x units lives in VGPRs for the whole sequence (it
//    never touches HBM); c_{t-1} and the saved gates S_t are read once (register ring,
//    two row tiles ahead); the cell backward of tile r-1 runs in fp32 micro-stages inside tile
//    r's MFMA loop; DG_t is written once with 16-B write-through (sc1) stores (lane pairs
//    exchange halves by DPP so each store is a whole 16-B (row, 2 units) run).
//  * SPLIT-PHASE hand-off (round 5). Batch rows are independent, so row tile r of step t
//    needs DG_{t+1} only of ITS rows — written by the row block's NB workgroups while they
//    ran tile r of the previous step, most of a step earlier. The NRT row tiles form NG groups
//    of GS tiles with one arrival counter each (persistent_sync.h): a workgroup publishes a
//    group (its waves drained the group's DG stores, workgroup barrier, one lane's agent-scope
//    add) a few tiles after the group's last tile, and every wave polls the counter of the
//    group its NEXT first-of-group tile needs two tiles ahead (one sc1 load, no spin). If the
//    poll matched, the wave streams that tile's A pieces in the previous tile's loop as for
//    any other tile — across the step boundary too: tile 0 of step t-1 is fetched during
//    tile NRT-1 of step t — else (a lagging peer) it waits at that tile (bounded spin) and
//    fetches it then. The round-4 kernel instead stopped every step: drain, barrier, add,
//    poll the whole row block, acquire, then fetch tile 0 (timeline: 4.2 us of a 28 us step).
//  * visibility (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH.md "Valid forms",
//    table row 1): every DG byte is stored sc1 by its producer, every storing wave waits for
//    its stores before the workgroup barrier behind which one lane adds to the counter, every
//    consumer wave polls the counter with an sc1 load itself and only then issues its A
//    loads, all with sc1 (the LDS-DMA form of the validated sc1 load-to-register: same
//    buffer_load path, L1 bypassed), so no acquire (L1 invalidate) is needed.
//  * every spin is bounded; a failing wave records why and runs on without waiting (results
//    garbage, the STAT block says so), so nothing can hang.
// Step T-1 (dh from the regression head) is lstm_bwd_last_kernel in lstm.hip.
#pragma once
// diagnostic builds: WELLFLOW_DIAG_BUILD=1 instantiates every timing variant, =N or =N,M,..
// only those WELLFLOW_PF_DBG values (fewer instantiations, minutes less to build)
#ifdef WF_DIAG
#ifndef WF_DIAG_SET
#define WF_DIAG_SET 0
#endif
#ifndef WF_DIAG_SET_DEFINED
#define WF_DIAG_SET_DEFINED
namespace wf {
constexpr int kDiagSet[] = {WF_DIAG_SET};
constexpr bool diag_variant(int v) {
  for (int x : kDiagSet)
    if (x == 0 || x == v) return true;
  return false;
}
}  // namespace wf
#endif
#define WF_DV(v) (::wf::diag_variant(v))
#endif
#include <cstdlib>

#include "gemm_core.h"
#include "kernels.h"
#include "lstm_layout.h"
#include "persistent_guard.h"
#include "persistent_launch.h"
#include "persistent_sync.h"

namespace wf {

namespace {
constexpr unsigned PB_SPIN_LIMIT = 1u << 21;
constexpr int PB_MAX_RT = 16;  // row tiles per workgroup (dc carry in registers: 4 VGPRs each)
// empty volatile asm redefining the value ("+v"): its producer stays above this point and its
// consumers below it (lstm_persistent.hip uses the same pins)
template <typename A> __device__ __forceinline__ void pin(A& a) { asm volatile("" : "+v"(a)); }
template <typename A, typename B> __device__ __forceinline__ void pin(A& a, B& b) {
  asm volatile("" : "+v"(a), "+v"(b));
}
}  // namespace

// Row tiles per hand-off group. A group's DG stores are known complete three tiles after its
// last tile (the stores of tile r issue in tile r+1's loop; a tile-top wait covers them two
// tiles later), and its first tile is polled two tiles before it runs, so a group must leave
// NRT - GS - 4 >= 0 tiles between its publish and its next poll: 8 of 16 (slack 4), 2 of 8
// (slack 2). NRT = 4 runs as one group: the old per-step hand-off (every poll falls back).
constexpr int pb_group_size(int nrt) { return nrt >= 16 ? 8 : (nrt >= 8 ? 2 : nrt); }

// KT = H / 32 k-tiles per wave (each wave's K quarter of G = 4H is H wide); NRT row tiles
// of 16 rows per workgroup (compile-time: the row-tile loop is fully unrolled so the dc
// carry, the prefetch rings and every vmcnt below are static).
// DBG (WF_DIAG timing-only builds, results wrong): 2 no MFMA, 16 no A loads after tile 1,
// 32 timeline (s_memrealtime stamps of step PB_STAMP_S, wave 0 lane 0 of every workgroup,
// into sync + 4096 words, 128 per workgroup; tools/pb_timeline.py).
// an A source: the buffer resource (MUBUF LDS-DMA) and the plain pointer (global_load_lds)
struct ASrc {
  __amdgpu_buffer_rsrc_t r;
  const char* p;
};

template <int KT, int NRT, int DBG = 0>
__global__ __launch_bounds__(256, 1) void lstm_bwd_persistent_kernel(
    const bf16_t* __restrict__ WhhT, const bf16_t* __restrict__ Cst, const bf16_t* __restrict__ S,
    bf16_t* __restrict__ DG, const float* __restrict__ dcarry, unsigned* __restrict__ sync,
    unsigned* __restrict__ stat, LstmDims d) {
  constexpr int H = 32 * KT, G = 4 * H, NB = H / 64, HB = H / 16;
  constexpr int KS = KT / 2;             // 64-wide k-steps per wave per row tile
  constexpr int GS = pb_group_size(NRT), NG = NRT / GS;
  constexpr bool GLDS = (DBG & 64) != 0;  // A pieces by global_load_lds (A/B; see issue_a)
  static_assert(NG <= kPSyncMaxGroups && NRT % GS == 0, "hand-off groups");
  static_assert(NG == 1 || (GS >= 2 && NRT - GS - 4 >= 0), "a group must publish before its next poll");
  constexpr int WSLOT = 16 * KT * 64;    // bytes of one wave's A tile: 16 rows x H k (bf16)
  constexpr int RING = 4 * 2 * WSLOT;    // [wave][2 slots]
  // partial sums [parity][src wave][rotation slot j][lane] x 16 B: wave w multiplies unit tile
  // (w + j) & 3 into acc[j], so its own tile is always acc[0] (no per-wave select) and slot j
  // of wave w holds unit tile (w + j) & 3 for the wave that owns it
  constexpr int RED = RING;
  // slots [p][w][0] of RED are never written (the own tile stays in registers): [0][0][0]
  // holds the epoch / started ordinal broadcast, [0][1][0] the per-wave failed words
  constexpr int BCAST = RED + (0 * 16 + 0 * 4 + 0) * 1024;
  constexpr int FAILW = RED + (0 * 16 + 1 * 4 + 0) * 1024;
  // ONE static LDS object (see lstm_persistent.hip: with several, the waitcnt pass guards LDS
  // accesses behind the LDS-DMA with vmcnt(0)); LDS writes go through inline asm.
  __shared__ __attribute__((aligned(16))) char smem[RED + 2 * 16 * 1024];
  typedef __attribute__((address_space(3))) char lds_char;
  const unsigned lds0 = (unsigned)(uintptr_t)((lds_char*)smem);

  const int Bp = fn_rows(d.B);
  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int m = L / NB, n = L % NB;
  const int row0 = m * 16 * NRT + d.row_off;  // row_off: sub-batch origin (launcher)
  const int ue = n * 64 + wid * 16 + l15;  // unit of this lane's cell backward
  const bool even = (l15 & 1) == 0;
  // production objects keep only the test hook bit (kDbgMask, persistent_guard.h)
  const int dbg = d.dbg & kDbgMask;
  ps_u32* rbw = psync_rb(sync, m);
  ps_u32* err = rbw + kPSyncErr;
  const unsigned spin_limit = d.spin_limit ? d.spin_limit : PB_SPIN_LIMIT;
  // (dbg bit 21, tests: an unreachable target, so every poll fails and the bounded spin trips)
  const unsigned force = ((dbg >> 21) & 1u) << 30;
  constexpr int PB_STAMP_S = 10;
  unsigned long long* stamps = reinterpret_cast<unsigned long long*>(sync + 4096) + blockIdx.x * 128;
  auto stamp = [&](int s, int slot) {
    if constexpr ((DBG & 32) != 0) {
      if (s == PB_STAMP_S && threadIdx.x == 0) stamps[slot] = __builtin_amdgcn_s_memrealtime();
    }
  };

  // completion guard (persistent_guard.h) and this launch's epoch (persistent_sync.h)
  if (threadIdx.x == 0) {
    const unsigned ord = pguard_start(stat, (unsigned)(d.T - 1));
    // a buffer last used by a launch of another (NRT, T, NB) fails loudly (persistent_sync.h)
    const unsigned sig = psync_sig(1u, (unsigned)NRT, (unsigned)d.T, (unsigned)NB);
    const unsigned bad = psync_check_sig(sync, sig);
    if (bad) {
      pguard_exit(stat, 0u, 5u, bad, 0u, sig, 0u, ord);
      pguard_sticky(stat);
    }
    const unsigned e = __hip_atomic_fetch_add(rbw + kPSyncStart, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) / NB;
    asm volatile("ds_write_b64 %0, %1" ::"v"(lds0 + BCAST), "v"((unsigned long long)e | ((unsigned long long)ord << 32))
                 : "memory");
    asm volatile("ds_write_b32 %0, %1" ::"v"(lds0 + BCAST + 8), "v"(bad) : "memory");
  }
  // ---- prologue: stationary W_hh^T fragments (B operand: lane = unit col l15, k 8g..8g+7)
  bf16x8 w[KT][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16_t* wr = WhhT + (size_t)(n * 64 + ((wid + j) & 3) * 16 + l15) * G + wid * H + 8 * g;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) w[kt][j] = *reinterpret_cast<const bf16x8*>(wr + 32 * kt);
  }
  // dc carry of step T-1 (lstm_bwd_last_kernel): registers for the whole sequence
  f32x4 dcr[NRT];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
    dcr[rt] = *reinterpret_cast<const f32x4*>(dcarry + fn_block(row0 + rt * 16, ue, H) * 256 + lane * 4);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  unsigned long long eo;
  unsigned sigbad;
  asm volatile("ds_read_b64 %0, %2\n\tds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(eo), "=&v"(sigbad)
               : "v"(lds0 + BCAST), "v"(lds0 + BCAST + 8)
               : "memory");
  const unsigned epoch = __builtin_amdgcn_readfirstlane((unsigned)eo);
  const unsigned ord = __builtin_amdgcn_readfirstlane((unsigned)(eo >> 32));
  const unsigned tag = epoch + 1u;
  // publishes of group g per launch: every step for groups published inside their step, all
  // but the last step for groups published at tile 1 of the next step (see pub_tile below)
  auto pub_rt = [](int gg) { return (gg + 1) * GS + 2; };  // global tile index of group gg's publish
  auto group_base = [&](int gg) -> unsigned {
    const bool in_step = NG == 1 || pub_rt(gg) <= NRT - 1;
    return epoch * (unsigned)NB * (unsigned)(in_step ? d.T - 1 : d.T - 2);
  };
  // arrivals group gg must show before step sg reads it: all NB workgroups published it for
  // steps 0 .. sg-1
  auto target = [&](int gg, int sg) { return group_base(gg) + (unsigned)(NB * sg) + force; };
  // uniform: this wave failed a hand-off or the signature check (runs on, never waits again)
  unsigned failed = __builtin_amdgcn_readfirstlane(sigbad) != 0u ? 1u : 0u;

  // ---- per-lane constant offsets
  // A (DG_{t+1}) staging: one LDS-DMA instruction = 8 rows x 128 B (full lines) of the wave's
  // K quarter; LDS image per 64-k step: [16 rows][8 x 16-B chunks], chunk c of row r in slot
  // c ^ ((r >> 1) & 7), so the fragment reads below are conflict-free (gemm_core.h K_CONTIG);
  // the swizzle moves onto the per-lane SOURCE address (the DMA writes LDS lane-linearly).
  const int dr = lane >> 3;  // row within the 8-row half written by this lane
  const int a_src = dr * G + wid * H + 8 * ((lane & 7) ^ ((dr >> 1) & 7));          // h = 0 (rows 0-7)
  const int a_src1 = (8 + dr) * G + wid * H + 8 * ((lane & 7) ^ (((8 + dr) >> 1) & 7));  // h = 1
  const int a_vo = a_src * 2, a_vo1 = a_src1 * 2;
  const unsigned a_lds = lds0 + wid * 2 * WSLOT;  // this wave's ring
  int fa[2];  // fragment byte offsets inside a 64-k step image, k-tile half 0 / 1
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) fa[hf] = l15 * 128 + (((4 * hf + g) ^ ((l15 >> 1) & 7)) << 4);
  const int s_lane = ue / 16 * 1024 + lane * 8;                     // FN S first half (block column ue>>4)
  const int c_lane = ue / 16 * 256 + lane * 4;                      // FN C slot
  const int ue2 = even ? ue : ue - 1;                               // first unit of this lane's 16-B run
  const int st_lane = ((4 * g + (even ? 0 : 1)) * G + 4 * ue2) * 2;  // byte offset (row 4g + r0, col 4*ue2)
  const size_t s_row = (size_t)(row0 >> 4) * HB * 1024 + s_lane, c_row = (size_t)(row0 >> 4) * HB * 256 + c_lane;

  // saved gates + c_{t-1} (HBM): 4-slot register ring, row tile rt in slot rt % 4 (NRT % 4 == 0,
  // so the slots line up across steps), issued two tiles ahead RIGHT AFTER the last A piece of
  // the current tile's loop: vmcnt completes in issue order, so an HBM load issued before an
  // A piece would hold that piece's wait for the whole HBM latency. The last two tiles of a
  // step prefetch tiles 0 and 1 of the next step (they do not depend on the hand-off). No
  // register of an in-flight load is ever moved.
  // Every address below is buffer-resource based: a 32-bit per-lane constant (s_vo / c_vo /
  // a_src) plus scalar (per step / per tile) parts, so the fully unrolled tile loop keeps no
  // per-tile 64-bit addresses live in VGPRs.
  const int s_vo = (int)(s_row * 2), c_vo = (int)(c_row * 2);
  // c_{t-1}: 4 bf16 per lane (the forward stores the cell-state history in bf16: half the
  // bytes of fp32 on both the forward's store and this read stream)
  typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
  u32x4 sq0[4], sq1[4];
  u32x2_t cq[4];
  auto cval = [&](int kp, int r) {  // c_{t-1} of row r (0..3) in ring slot kp
    const unsigned wv = cq[kp][r >> 1];
    return __uint_as_float((r & 1) ? (wv & 0xffff0000u) : (wv << 16));
  };
  auto load_sc = [&](int t, auto rc, auto slot) {
    constexpr int RT = decltype(rc)::value, Q = decltype(slot)::value;
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(S) + (size_t)t * Bp * G, 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(Cst) + (size_t)t * Bp * H, 0, 0x7FFFFFFF, 0x00020000);
    constexpr int SO = RT * HB * 1024 * 2, CO = RT * HB * 256 * 2;
    // nt on the read-once streams
    sq0[Q] = __builtin_amdgcn_raw_buffer_load_b128(sr, s_vo, SO, 2);
    sq1[Q] = __builtin_amdgcn_raw_buffer_load_b128(sr, s_vo + 2 * kFnSHalf, SO, 2);  // second half
    cq[Q] = __builtin_amdgcn_raw_buffer_load_b64(cr, c_vo, CO, 2);
  };
  // A tile TI of the step whose A resource is `ar` -> ring slot TI & 1; piece i = k-step i / 2,
  // rows 8 * (i % 2) .. of the wave's K quarter, 1 KB, sc1 (the hand-off's consumer side)
  auto issue_a = [&](const ASrc& ar, auto tc, auto ic) {
    constexpr int TI = decltype(tc)::value, i = decltype(ic)::value, ks = i / 2, hf = i % 2;
    if constexpr ((DBG & 16) != 0) {
      if (TI > 1) return;
    }
    const unsigned dst = a_lds + (TI & 1) * WSLOT + ks * 2048 + hf * 1024;
    if constexpr (GLDS) {
      // global_load_lds (round 6, DBG 64 A/B): same bytes, same LDS image, sc1. Tried because
      // the probe charged the MUBUF form ~2x its issue time beside MFMAs; in the real kernel it
      // measured SLOWER (1.492 vs 1.466 ms, profiles/r6/diag/glds.txt): MUBUF stays
      const char* src = ar.p + (hf ? a_vo1 : a_vo) + TI * 16 * G * 2 + ks * 128;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(uintptr_t)dst, 16, 0, 16 /* sc1 */);
    } else {
      // (the instruction offset would also move the LDS address: the k-step goes into soffset)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ar.r, (lds_void*)(uintptr_t)dst, 16, hf ? a_vo1 : a_vo,
                                               TI * 16 * G * 2 + ks * 128, 0, 16);
    }
  };
  auto a_rsrc_of = [&](int tt) -> ASrc {  // A of the step with t = tt: DG_{tt+1}, this row block
    const bf16_t* b = DG + ((size_t)(tt + 1) * d.B + row0) * G;
    return ASrc{__builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(b), 0, 0x7FFFFFFF, 0x00020000),
                reinterpret_cast<const char*>(b)};
  };

  // sc1 poll of a group counter: one uniform load (every lane, one address). Inline asm, so it
  // stays where it is written (the compiler sinks the S / c buffer loads to the end of the
  // loop, behind the DG stores; a tracked poll there made its first use wait for those stores)
  // and the tile-top wait that covers it names its register (poll_wait).
  auto poll = [&](int gg) {
    unsigned v;
    const unsigned* pa = sync + kPSyncHead + kPSyncRowBlock * m + kPSyncGroup + gg;
    asm volatile("global_load_dword %0, %1, off sc1" : "=v"(v) : "v"(pa) : "memory");
    return v;
  };
  // blocking wait of this wave for group gg before step sg (slow path); a failure is recorded
  // once and turns every later wait of the wave into a no-op
  auto wait_group = [&](int gg, int sg) {
    if (failed) return;
    unsigned seen_cnt = 0, seen_err = 0;
    const unsigned tg = target(gg, sg);
    const unsigned why = psync_wait(rbw + kPSyncGroup + gg, err, tg, tag, spin_limit, stat, &seen_cnt, &seen_err);
    if (why != 0) {
      failed = 1;
      if (lane == 0) pguard_exit(stat, (unsigned)sg, why, seen_err, seen_cnt, tg, (unsigned)gg, ord);
    }
  };
  auto publish = [&](int gg) {  // behind a workgroup barrier every wave reached after its stores drained
    if (threadIdx.x == 0) __hip_atomic_fetch_add(rbw + kPSyncGroup + gg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  constexpr int NSC = 3;  // S / c loads per tile
  constexpr int NST = 2;  // DG stores per tile
  load_sc(d.T - 2, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
  load_sc(d.T - 2, std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
  {  // A(0) of the first step: DG_{T-1} was written by the previous kernel (lstm_bwd_last_kernel)
    const ASrc ar = a_rsrc_of(d.T - 2);
    static_for<0, 2 * KS>([&](auto ic) { issue_a(ar, std::integral_constant<int, 0>{}, ic); });
  }
  // fast[gg]: this wave already streamed the first tile of group gg (its poll matched two tiles
  // ahead); at step 0 every group is ready (DG_{T-1} comes from the previous kernel)
  unsigned fast[NG];
#pragma unroll
  for (int gg = 0; gg < NG; ++gg) fast[gg] = 1;
  unsigned pv = 0;  // the outstanding poll's value (uniform)

  // dh partial of the previous tile, own unit tile (the other three go through LDS)
  f32x4 dho = f32x4{0.f, 0.f, 0.f, 0.f};
  // where the other waves' partials of this wave's unit tile sit: slot j of wave (wid - j) & 3
  // (+ parity * 16 KB as an immediate)
  unsigned rdj[4];
#pragma unroll
  for (int j = 1; j < 4; ++j) rdj[j] = lds0 + RED + ((wid - j) & 3) * 4096 + j * 1024 + lane * 16;
  const unsigned wr_base = lds0 + RED + wid * 4096 + lane * 16;  // red[.][wid][.][lane]

  for (int s = 0; s < d.T - 1; ++s) {
    const int t = d.T - 2 - s;
    const bool last_step = s == d.T - 2;
    stamp(s, 0);
    const ASrc a_rsrc = a_rsrc_of(t);
    const ASrc an_rsrc = a_rsrc_of(t > 0 ? t - 1 : t);  // next step's A (DG_t)
    const __amdgpu_buffer_rsrc_t dg_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(DG + (size_t)t * d.B * G, 0, 0x7FFFFFFF, 0x00020000);
    const int st_base = row0 * G * 2 + st_lane;

    // Cell backward parts 7 (lane-pair exchange) and 8 (the two DG stores) of row tile RTp.
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x4 dhp = f32x4{0.f, 0.f, 0.f, 0.f};
    unsigned ev[4][2];
    f32x4 enk;
    u32x4 elo, ehi;
    auto epi = [&](auto rpc, auto partc) {
      constexpr int RTp = decltype(rpc)::value, part = decltype(partc)::value;
      if constexpr (part == 7) {
        dcr[RTp] = enk;
        // lane pair (2i, 2i+1) = units (u, u+1): the even lane stores rows 0, 2 and the odd
        // lane rows 1, 3 of both units, each a 16-B run [4 gates of u | 4 gates of u+1]
        const unsigned snd[4] = {even ? ev[1][0] : ev[0][0], even ? ev[1][1] : ev[0][1],
                                 even ? ev[3][0] : ev[2][0], even ? ev[3][1] : ev[2][1]};
        unsigned o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          o[i] = (unsigned)__builtin_amdgcn_mov_dpp((int)snd[i], 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
        if (even) {
          elo = u32x4{ev[0][0], ev[0][1], o[0], o[1]};  // row 4g + 0: units u, u+1
          ehi = u32x4{ev[2][0], ev[2][1], o[2], o[3]};  // row 4g + 2
        } else {
          elo = u32x4{o[0], o[1], ev[1][0], ev[1][1]};  // row 4g + 1: units u-1, u
          ehi = u32x4{o[2], o[3], ev[3][0], ev[3][1]};  // row 4g + 3
        }
      } else if constexpr (part == 8) {
        constexpr int SOFF = RTp * 16 * G * 2;
        // sc1 (write-through): the hand-off's producer side
        __builtin_amdgcn_raw_buffer_store_b128(elo, dg_rsrc, st_base, SOFF, 16);
        __builtin_amdgcn_raw_buffer_store_b128(ehi, dg_rsrc, st_base, SOFF + 2 * G * 2, 16);
      }
    };

    // The cell backward as 64 micro-stages in scalar fp32, one per MFMA of the next tile's loop
    // (at most two plain ops or one transcendental: what a 16x16x32 MFMA leaves free of its
    // 16 issue cycles; packed fp32 costs more issue beside MFMAs than two scalar ops).
    // Stage q < 60: rows 2p, 2p+1 (p = q / 30) in flight together, stage (q % 30) / 2 of row
    // 2p + (q & 1); q = 60: lane-pair exchange (part 7); q = 62: DG stores (part 8). Every
    // stage pins its values with empty "+v" asm, so the compiler can neither sink the math
    // below the MFMAs nor hoist it above them (it had gathered each part into one clump).
    struct BRow {
      unsigned sa, sb;
      float i, f, g, o, x, tc, eq, dc, nk, a, tq, u, di, dg, df, e;
      unsigned p0, p1;
    };
    BRow brow[2];
    auto bstage = [&](auto rpc, auto qc) {
      constexpr int RTp = decltype(rpc)::value, q = decltype(qc)::value, Kp = RTp % 4;
      if constexpr (q < 60) {
        constexpr int r = 2 * (q / 30) + (q & 1), st = (q % 30) / 2;
        BRow& b = brow[q & 1];
        if constexpr (st == 0) {
          const u32x4 sv = r < 2 ? sq0[Kp] : sq1[Kp];  // row r: (i|f), (g|o)
          b.sa = sv[2 * (r & 1)];
          b.sb = sv[2 * (r & 1) + 1];
          b.i = __uint_as_float(b.sa << 16);
          b.f = __uint_as_float(b.sa & 0xffff0000u);
          pin(b.i, b.f);
          pin(b.sb);
        } else if constexpr (st == 1) {
          b.g = __uint_as_float(b.sb << 16);
          b.o = __uint_as_float(b.sb & 0xffff0000u);
          pin(b.g, b.o);
        } else if constexpr (st == 2) {  // c_t = fma(f, c_{t-1}, i g) as the forward rounds it
          b.x = b.i * b.g;
          b.x = __builtin_fmaf(b.f, cval(Kp, r), b.x);
          pin(b.x);
        } else if constexpr (st == 3) {
          b.x = b.x * 2.8853900817779268f;  // exp(2 c) = 2^(2 log2(e) c)
          pin(b.x);
        } else if constexpr (st == 4) {
          b.x = __builtin_amdgcn_exp2f(b.x);
          pin(b.x);
        } else if constexpr (st == 5) {
          b.x = b.x + 1.f;
          pin(b.x);
        } else if constexpr (st == 6) {
          b.x = __builtin_amdgcn_rcpf(b.x);
          pin(b.x);
        } else if constexpr (st == 7) {  // tanh(c_t); dh o
          b.tc = 1.f - 2.f * b.x;
          b.eq = dhp[r] * b.o;
          pin(b.tc, b.eq);
        } else if constexpr (st == 8) {  // dc = dh o (1 - tanh^2) + carry
          b.dc = 1.f - b.tc * b.tc;
          b.dc = __builtin_fmaf(b.eq, b.dc, dcr[RTp][r]);
          pin(b.dc);
        } else if constexpr (st == 9) {
          b.nk = b.dc * b.f;  // carry to step t-1
          b.a = b.dc * b.i;
          pin(b.nk, b.a);
        } else if constexpr (st == 10) {
          b.tq = b.a * b.g;
          b.u = b.nk * cval(Kp, r);
          pin(b.tq, b.u);
        } else if constexpr (st == 11) {
          b.di = b.tq - b.tq * b.i;  // dc g i (1 - i)
          b.dg = b.a - b.tq * b.g;   // dc i (1 - g^2)
          pin(b.di, b.dg);
        } else if constexpr (st == 12) {
          b.df = b.u - b.u * b.f;  // dc c_{t-1} f (1 - f)
          b.e = b.eq * b.tc;
          pin(b.df, b.e);
        } else if constexpr (st == 13) {
          const float dO = b.e - b.e * b.o;  // dh tanh(c) o (1 - o)
          b.p0 = pk_bf16(b.di, b.df);
          b.p1 = pk_bf16(b.dg, dO);
          pin(b.p0, b.p1);
        } else {
          ev[r][0] = b.p0;
          ev[r][1] = b.p1;
          enk[r] = b.nk;
        }
      } else if constexpr (q == 60) {
        epi(rpc, std::integral_constant<int, 7>{});
      } else if constexpr (q == 62) {
        epi(rpc, std::integral_constant<int, 8>{});
      }
    };

    // K-split partial exchange, deferred by one tile: tile r writes its 3 foreign partials to
    // red[r & 1] at its end and runs on; tile r+1's loop passes a barrier after its first
    // k-tile (the writes drained by that k-tile's lgkmcnt wait), issues the partial reads, and
    // sums them at k-tile 1 (so their LDS latency hides under MFMAs). The last tile of a step
    // exchanges at once and runs its cell backward there (the next step's tile 0 needs the
    // carry, and the step's last group is published from it).
    static_for<0, NRT>([&](auto rc) {
      constexpr int RT = decltype(rc)::value, P = RT & 1;
      constexpr bool GFIRST = RT % GS == 0;
      constexpr int GRT = RT / GS;
      // ---- first tile of a group whose poll did not match two tiles ago: wait, then fetch
      if constexpr (GFIRST && NG > 1) {
        if (!fast[GRT]) {
          stamp(s, 1);
          wait_group(GRT, s);
          static_for<0, 2 * KS>([&](auto ic) { issue_a(a_rsrc, rc, ic); });
          wait_vmcnt<0>();
        }
      } else if constexpr (NG == 1 && RT == 0) {
        if (s > 0) {  // one group: the old per-step hand-off (published at the previous step's end)
          wait_group(0, s);
          static_for<0, 2 * KS>([&](auto ic) { issue_a(a_rsrc, rc, ic); });
          wait_vmcnt<0>();
        }
      }
      // ---- wait for A(RT): its pieces were issued in the first half of tile RT-1's MFMA loop;
      // after the last one came tile RT-1's S / c loads (of tile RT+1 or of the next step) and
      // tile RT-2's DG stores (epilogue part 8, if RT-1 > 0), which may stay in flight; at tile
      // 0 the previous step's last two tiles' stores too
      if constexpr (RT == 0) {
        if (s == 0)
          wait_vmcnt<0>();
        else
          wait_vmcnt<NSC + 2 * NST>();
      } else if constexpr (RT == 1) {
        wait_vmcnt<NSC>();
      } else if constexpr (NG > 1 && (RT + 1 == NRT || (RT + 1) % GS == 0)) {
        // the poll issued in the previous loop is older than its S / c loads and DG stores:
        // this wait covers it (the operand keeps its consumers below the wait)
        asm volatile("s_waitcnt vmcnt(%1)" : "+v"(pv) : "n"(NSC + NST) : "memory");
      } else {
        wait_vmcnt<NSC + NST>();
      }
      stamp(s, 2 + 5 * RT);
      // ---- the poll issued in the previous tile's loop decides whether this tile's loop
      // streams the next group's first tile (RT + 1 = first of a group at this step, or tile 0
      // of the next step)
      constexpr bool NEXT_GFIRST = NG > 1 && (RT + 1 == NRT || (RT + 1) % GS == 0);
      constexpr int NGRP = (RT + 1 == NRT) ? 0 : (RT + 1) / GS;
      if constexpr (NEXT_GFIRST) {
        if (RT + 1 == NRT) {
          fast[NGRP] = last_step ? 0u : (failed | (psync_reached(__builtin_amdgcn_readfirstlane(pv), target(NGRP, s + 1)) ? 1u : 0u));
        } else {
          fast[NGRP] = s == 0 ? 1u : (failed | (psync_reached(__builtin_amdgcn_readfirstlane(pv), target(NGRP, s)) ? 1u : 0u));
        }
      }
      const unsigned cur = a_lds + P * WSLOT;

      f32x4 acc[4];  // written first by k-tile 0's MFMAs (src C = 0)
      f32x4 pr[4];
      // A fragments two k-tiles ahead (3-register ring): with one ahead (4 MFMAs, ~64 cycles)
      // the ds_read latency under the concurrent LDS-DMA traffic was partly exposed at every
      // k-tile. LDS returns in order; the waits count the reads younger than k-tile kt's:
      // r_{kt+1}, r_{kt+2} and, at kt = 1, the 3 partial-sum reads issued at the end of kt = 0
      // (RT > 0); k-tile KSUM waits for those partials too (they are summed there).
      bf16x8 a[3];
      asm volatile("ds_read_b128 %0, %1" : "=v"(a[0]) : "v"(cur + fa[0]) : "memory");
      if constexpr (KT > 1)
        asm volatile("ds_read_b128 %0, %1" : "=v"(a[1]) : "v"(cur + fa[1]) : "memory");
      static_for<0, KT>([&](auto kc) {
        constexpr int kt = decltype(kc)::value;
        (void)acc;  // odr-use outside the asm operands: clang does not capture them implicitly
        (void)w;
        (void)pr;
        if constexpr (kt + 2 < KT)
          asm volatile("ds_read_b128 %0, %1 offset:%2"
                       : "=v"(a[(kt + 2) % 3])
                       : "v"(cur + fa[(kt + 2) & 1]), "i"(((kt + 2) >> 1) * 2048)
                       : "memory");
        // k-tile whose top sums the partials: 2, or 1 where the cell backward's first use of dh
        // (micro-stage 7) already falls into k-tile 1 (KT = 4, H = 128)
        constexpr int KSUM = KT >= 8 ? 2 : 1;
        constexpr int YOUNGER = (kt + 1 < KT ? 1 : 0) + (kt + 2 < KT ? 1 : 0) + (RT > 0 && kt == 1 && KSUM == 2 ? 3 : 0);
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(YOUNGER) : "memory");
        if constexpr (RT > 0 && kt == KSUM) {
          // the wait above drained the partial reads issued at k-tile 0 (LDS returns in order:
          // only the fragment reads after them are younger): tie them to it, then the previous tile's dh
          asm volatile("" : "+v"(pr[1]), "+v"(pr[2]), "+v"(pr[3]));
          dhp = dho + ((pr[1] + pr[2]) + pr[3]);
        }
        static_for<0, 4>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if constexpr (!(DBG & 2)) {
            if constexpr (kt == 0)
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc[j]) : "v"(a[kt % 3]), "a"(w[kt][j]));
            else
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(a[kt % 3]), "a"(w[kt][j]));
          }
          if constexpr (RT > 0) {
            // stage instances [qlo, qhi) after MFMA slot m, from k-tile 1 on (dh of the
            // previous tile is summed at the top of k-tile 1)
            constexpr int S = 4 * KT - 4, m = kt * 4 + j - 4;
            if constexpr (m >= 0) {
              constexpr int qlo = (m * 64 + S - 1) / S, qhi = ((m + 1) * 64 + S - 1) / S;
              static_for<qlo, qhi>([&](auto qc) { bstage(std::integral_constant<int, RT - 1>{}, qc); });
            }
          }
        });
        // two A pieces of the next tile per k-tile over the first half of the loop: the vector-
        // memory queue drains under the MFMAs instead of blocking the wave before them, and the
        // last piece lands well before the next tile needs it. The next tile is tile 0 of the
        // next step at RT = NRT - 1, and a group's first tile only when its poll matched.
        if constexpr (2 * kt < KT) {
          if constexpr (RT + 1 == NRT) {
            if constexpr (NG > 1) {
              if (fast[0] && !last_step) {
                issue_a(an_rsrc, std::integral_constant<int, 0>{}, std::integral_constant<int, 2 * kt>{});
                issue_a(an_rsrc, std::integral_constant<int, 0>{}, std::integral_constant<int, 2 * kt + 1>{});
              }
            }
          } else if constexpr ((RT + 1) % GS == 0) {
            if (fast[(RT + 1) / GS]) {
              issue_a(a_rsrc, std::integral_constant<int, RT + 1>{}, std::integral_constant<int, 2 * kt>{});
              issue_a(a_rsrc, std::integral_constant<int, RT + 1>{}, std::integral_constant<int, 2 * kt + 1>{});
            }
          } else {
            issue_a(a_rsrc, std::integral_constant<int, RT + 1>{}, std::integral_constant<int, 2 * kt>{});
            issue_a(a_rsrc, std::integral_constant<int, RT + 1>{}, std::integral_constant<int, 2 * kt + 1>{});
          }
        }
        if constexpr (kt == KT / 2 - 1) {  // S / c of tile RT + 2 right after the last A piece
          __builtin_amdgcn_sched_barrier(0);
          // the poll for the first tile of the group two tiles ahead (after the A pieces: an
          // L2 round trip; before the S / c loads: HBM latency would hold it in the queue)
          constexpr bool POLL = NG > 1 && (RT + 2 == NRT || (RT + 2 < NRT && (RT + 2) % GS == 0));
          if constexpr (POLL) pv = poll(RT + 2 == NRT ? 0 : (RT + 2) / GS);
          if constexpr (RT + 2 < NRT)
            load_sc(t, std::integral_constant<int, RT + 2>{}, std::integral_constant<int, (RT + 2) % 4>{});
          else  // tiles 0 / 1 of the next step (t - 1; past step 0: a harmless reload, same count)
            load_sc(t > 0 ? t - 1 : t, std::integral_constant<int, RT + 2 - NRT>{},
                    std::integral_constant<int, (RT + 2) % 4>{});
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (RT > 0 && kt == 0) {
          // every wave's partial writes of tile RT-1 were drained by its lgkmcnt wait above, and
          // every wave's DG stores older than its tile-top wait have completed
          __builtin_amdgcn_s_barrier();
          // publish a group whose last DG stores every wave has now drained: in-step groups at
          // tile (last + 3); groups whose publish tile falls past the step end (the step's last
          // group among them) at tile 1 of the next step
          static_for<0, NG>([&](auto gc) {
            constexpr int gg = decltype(gc)::value;
            if constexpr (NG > 1) {
              constexpr int pr_t = (gg + 1) * GS + 2;
              if constexpr (pr_t <= NRT - 1 && RT == pr_t) publish(gg);
              if constexpr (pr_t > NRT - 1 && RT == 1) {
                if (s > 0) publish(gg);
              }
            }
          });
          static_for<1, 4>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            (void)pr;
            (void)rdj;
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(pr[j]) : "v"(rdj[j]), "i"(((RT - 1) & 1) * 16384)
                         : "memory");
          });
        }
        // the MFMAs above are inline asm, so the compiler knows neither their latency nor that
        // they still read this fragment: keep its registers allocated until here, so no VALU
        // result of the interleaved epilogue can land in them while the MFMAs are in flight
        asm volatile("" ::"v"(a[kt % 3]));
      });
      // VALU / LDS reads of MFMA results: cover the pipeline (nothing is padded after asm)
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((DBG & 32) != 0) {  // MFMA completion: consume a result before stamping
        float sink = acc[3][3];
        asm volatile("" ::"v"(sink));
        stamp(s, 3 + 5 * RT);
      }

      // ---- K-split partials -> red[P][wid][1..3] (the own unit tile stays in registers: dho)
      dho = acc[0];
#pragma unroll
      for (int j = 1; j < 4; ++j)
        asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(wr_base), "v"(acc[j]), "i"(P * 16384 + j * 1024) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      stamp(s, 4 + 5 * RT);
      if constexpr (RT + 1 == NRT) {  // last tile: exchange now, drain its cell backward
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        static_for<1, 4>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          (void)acc;
          (void)rdj;
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(acc[j]) : "v"(rdj[j]), "i"(P * 16384) : "memory");
        });
        // the wait takes the accumulators as operands: the compiler sees inline-asm outputs as
        // ready at once and would otherwise schedule the sum between the reads and the wait
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]) :: "memory");
        dhp = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        stamp(s, 5 + 5 * RT);
        static_for<0, 64>([&](auto qc) { bstage(std::integral_constant<int, RT>{}, qc); });
        if constexpr (NG == 1) {  // one group: publish the whole step now (drain, barrier, add)
          wait_vmcnt<0>();
          __builtin_amdgcn_s_barrier();
          publish(0);
        }
      }
      stamp(s, 6 + 5 * RT);
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  // completion count (DONE vs EXPECT, persistent_guard.h): only if no wave failed a hand-off
  wait_vmcnt<0>();
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds0 + FAILW + wid * 4), "v"(failed) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (threadIdx.x == 0) {
    u32x4 fw;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(fw) : "v"(lds0 + FAILW) : "memory");
    if ((fw[0] | fw[1] | fw[2] | fw[3]) == 0u) pguard_done(stat, (unsigned)(d.T - 1));
  }
}

template <int KT, int NRT>
static int launch_pb(const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S, bf16_t* DG, const float* dcarry,
                      unsigned* sync, unsigned* stat, int grid, LstmDims d, hipStream_t s) {
  const void* f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT>);
#ifdef WF_DIAG  // timing-only variants: diagnostic builds only (WELLFLOW_DIAG_BUILD=1)
  const void* const prod = f;
  if constexpr (KT == 16 && NRT == 16) {
    switch (d.dbg & 0xFFFFF) {
      case 2: if constexpr (WF_DV(2)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 2>); break;
      case 16: if constexpr (WF_DV(16)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 16>); break;
      case 32: if constexpr (WF_DV(32)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 32>); break;
      case 64: if constexpr (WF_DV(64)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 64>); break;
      default: break;
    }
  }
  // a requested variant that this build did not compile must not time the production kernel
  // under its name (bits 20-22 are runtime switches, not variants)
  if ((d.dbg & 0xFFFFF) != 0 && f == prod) return -(int)hipErrorInvalidDeviceFunction;
#endif
  void* args[] = {&WhhT, &Cst, &S, &DG, &dcarry, &sync, &stat, &d};
  return persistent_launch(f, grid, args, s);  // persistent_launch.h
}

}  // namespace wf
