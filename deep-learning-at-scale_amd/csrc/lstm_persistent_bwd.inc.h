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
//    two row tiles ahead); the cell backward of tile r-1 runs in packed fp32 inside tile r's
//    MFMA loop; DG_t is written once with 16-B write-through (sc1) stores (lane pairs
//    exchange halves by DPP so each store is a whole 16-B (row, 2 units) run).
//  * hand-off (cdna_hip_programming.md Guideline 16, recipe R1, as in the forward): every
//    wave drains its stores (vmcnt(0)), workgroup barrier, ONE lane adds to the row
//    block's arrival counter (agent scope); consumers poll relaxed with s_sleep, then ONE
//    agent-scope acquire, then the LDS-DMA loads of DG_{t+1}. Only the H/64 workgroups of one
//    row block depend on each other; every spin is bounded (error words 1 and sticky 0, all drain).
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

namespace wf {

namespace {
constexpr unsigned PB_SPIN_LIMIT = 1u << 21;
constexpr int PB_MAX_RT = 16;  // row tiles per workgroup (dc carry in registers: 4 VGPRs each)
typedef __attribute__((address_space(1))) unsigned gu32;
// empty volatile asm redefining the value ("+v"): its producer stays above this point and its
// consumers below it (lstm_persistent.hip uses the same pins)
template <typename A> __device__ __forceinline__ void pin(A& a) { asm volatile("" : "+v"(a)); }
template <typename A, typename B> __device__ __forceinline__ void pin(A& a, B& b) {
  asm volatile("" : "+v"(a), "+v"(b));
}
}  // namespace

// KT = H / 32 k-tiles per wave (each wave's K quarter of G = 4H is H wide); NRT row tiles
// of 16 rows per workgroup (compile-time: the row-tile loop is fully unrolled so the dc
// carry, the prefetch rings and every vmcnt below are static).
// DBG (timing-only builds, results wrong; WELLFLOW_PF_DBG at H = 512, NRT = 16):
// 1 no hand-off wait, 2 no MFMA, 4 no DG stores, 8 no S / c loads, 16 no A loads, 128 A
// always from row tile 0 (same bytes, L2-hot), 256 default-policy (not nt) S / c loads;
// 64 = plain (L2-resident) DG stores + agent release before the arrival add (correct results);
// 32 = timeline: s_memrealtime stamps of step PB_STAMP_S, wave 0 lane 0 of every workgroup,
// into sync + 4096 words (128 per workgroup; tools/pb_timeline.py).
template <int KT, int NRT, int DBG = 0>
__global__ __launch_bounds__(256, 1) void lstm_bwd_persistent_kernel(
    const bf16_t* __restrict__ WhhT, const bf16_t* __restrict__ Cst, const bf16_t* __restrict__ S,
    bf16_t* __restrict__ DG, const float* __restrict__ dcarry, unsigned* __restrict__ sync,
    unsigned* __restrict__ stat, LstmDims d) {
  constexpr int H = 32 * KT, G = 4 * H, NB = H / 64, HB = H / 16;
  constexpr int KS = KT / 2;             // 64-wide k-steps per wave per row tile
  constexpr bool MICRO = (DBG & 512) == 0;  // cell backward as per-MFMA micro-stages (bstage)
  constexpr int WSLOT = 16 * KT * 64;    // bytes of one wave's A tile: 16 rows x H k (bf16)
  constexpr int RING = 4 * 2 * WSLOT;    // [wave][2 slots]
  constexpr int RED = RING;              // partial sums [parity][src wave][unit tile][lane] x 16 B
  constexpr int FLAG = RED + (1 * 16 + 0 * 4 + 0) * 1024;  // slot [1][0][0]: never written (own tile)
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
  // this launch's error (word 1 in the round-2 layout A/B, PF_DBG bit 20); the sticky bit is
  // in the STAT block (persistent_guard.h)
  // production objects keep only the test hook bit (kDbgMask, persistent_guard.h): the
  // timing-only branches below fold away at compile time
  const int dbg = d.dbg & kDbgMask;
  gu32* err = (gu32*)(sync + ((dbg >> 20) & 1));
  gu32* cnt = (gu32*)(sync + 16 + 16 * m);
  const unsigned spin_limit = d.spin_limit ? d.spin_limit : PB_SPIN_LIMIT;
  constexpr int PB_STAMP_S = 10;
  unsigned long long* stamps = reinterpret_cast<unsigned long long*>(sync + 4096) + blockIdx.x * 128;
  auto stamp = [&](int s, int slot) {
    if constexpr ((DBG & 32) != 0) {
      if (s == PB_STAMP_S && threadIdx.x == 0) stamps[slot] = __builtin_amdgcn_s_memrealtime();
    }
  };

  // completion guard (persistent_guard.h): started / expected counts before any exit path
  unsigned ord = 0;
  if (threadIdx.x == 0) ord = pguard_start(stat, (unsigned)(d.T - 1));
  // ---- prologue: stationary W_hh^T fragments (B operand: lane = unit col l15, k 8g..8g+7)
  bf16x8 w[KT][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16_t* wr = WhhT + (size_t)(n * 64 + j * 16 + l15) * G + wid * H + 8 * g;
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
    if constexpr ((DBG & 8) != 0) {
      if (t < d.T - 2 || RT > 1) return;
    }
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(S) + (size_t)t * Bp * G, 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(Cst) + (size_t)t * Bp * H, 0, 0x7FFFFFFF, 0x00020000);
    constexpr int SO = RT * HB * 1024 * 2, CO = RT * HB * 256 * 2;
    // nt on the read-once streams (256: default policy; A/B within run-to-run noise)
    constexpr int NTA = (DBG & 256) ? 0 : 2;
    sq0[Q] = __builtin_amdgcn_raw_buffer_load_b128(sr, s_vo, SO, NTA);
    sq1[Q] = __builtin_amdgcn_raw_buffer_load_b128(sr, s_vo + 2 * kFnSHalf, SO, NTA);  // second half
    cq[Q] = __builtin_amdgcn_raw_buffer_load_b64(cr, c_vo, CO, NTA);
  };
  load_sc(d.T - 2, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
  load_sc(d.T - 2, std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});

  for (int s = 0; s < d.T - 1; ++s) {
    const int t = d.T - 2 - s;
    stamp(s, 0);
    if (s > 0) {
      // ---- publish step s-1 (every wave drained its DG stores) and wait for the row block
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // thread 0's view of the wait, kept for the exit record (persistent_guard.h)
      unsigned why = 0, seen_err = 0, seen_cnt = 0;
      // (dbg bit 21, tests: an unreachable target, so the bounded spin trips deterministically)
      const unsigned target = (unsigned)(NB * s) + (((dbg >> 21) & 1u) << 30);
      if (threadIdx.x == 0) {
        if constexpr ((DBG & 64) != 0) {  // plain DG stores: publish them with an agent release
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (!(DBG & 1) && (seen_cnt = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < target) {
          if ((seen_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u) {
            why = 1;
            break;
          }
          if (++spins > spin_limit) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pguard_sticky(stat);
            why = 2;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        // (dbg bit 22, WF_DIAG builds only, WELLFLOW_PF_DBG=4194304: TIMING ONLY, unsafe — no acquire, to price it)
        if (!((dbg >> 22) & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int ok = why == 0 ? 1 : 0;
        asm volatile("ds_write_b32 %0, %1" ::"v"(lds0 + FLAG), "v"(ok) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      int okv;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(okv) : "v"(lds0 + FLAG) : "memory");
      if (__builtin_amdgcn_readfirstlane(okv) != 1) {  // uniform
        if (lane == 0)
          pguard_exit(stat, (unsigned)s, wid != 0 ? 4u : (why != 0 ? why : 3u), seen_err, seen_cnt, target,
                      (unsigned)okv, ord);
        return;
      }
    }

    stamp(s, 1);
    const __amdgpu_buffer_rsrc_t a_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(DG + ((size_t)(t + 1) * d.B + row0) * G, 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t dg_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(DG + (size_t)t * d.B * G, 0, 0x7FFFFFFF, 0x00020000);
    const int st_base = row0 * G * 2 + st_lane;
    // A tile rt of this wave -> ring slot rt & 1: KS k-steps x 2 row halves, 1 KB each
    // piece i (k-step i / 2, rows 8 * (i % 2) ..) of A tile RT of this wave -> ring slot RT & 1
    auto issue_a = [&](auto rc, auto ic) {
      constexpr int RT = decltype(rc)::value, i = decltype(ic)::value, ks = i / 2, hf = i % 2;
      if constexpr ((DBG & 16) != 0) {
        if (RT > 1) return;
      }
      const unsigned dst = a_lds + (RT & 1) * WSLOT + ks * 2048 + hf * 1024;
      // (the instruction offset would also move the LDS address: the k-step goes into soffset)
      constexpr int RTS = (DBG & 128) ? 0 : RT;  // timing build 128: always row tile 0 (L2-hot lines)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_void*)(uintptr_t)dst, 16, hf ? a_vo1 : a_vo,
                                               RTS * 16 * G * 2 + ks * 128, 0, 0);
    };
    constexpr int NA = ((DBG & 16) != 0) ? 0 : 2 * KS;  // DMA instructions per A tile (= KT)
    constexpr int NSC = ((DBG & 8) != 0) ? 0 : 3;       // S / c loads per tile
    constexpr int NST = ((DBG & 4) != 0) ? 0 : 2;       // DG stores per tile
    static_assert(2 * KS == KT, "two A pieces per k-tile over the first half of the loop");
    (void)NA;
    static_for<0, 2 * KS>([&](auto ic) { issue_a(std::integral_constant<int, 0>{}, ic); });

    // Cell backward of row tile RTp (its dh in dhp, its saved gates / c_{t-1} in ring slot
    // RTp % 3, its carry in dcr[RTp]) in parts 1..EPI_PARTS, two rows at a time in packed fp32
    // (v_pk_fma / v_pk_mul: half the VALU issue of the scalar form), so that tile RTp + 1's
    // MFMA loop can issue one part per k-tile in the MFMAs' shadow (software pipeline).
    //   per row pair q: part 3q+1 gates, x = f c + i g, e = exp(2x); part 3q+2 tanh, dc, carry;
    //   part 3q+3 the four gate gradients, packed to bf16; part 7 lane-pair exchange; 8 stores.
    constexpr int EPI_PARTS = 8;
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x4 dhp = f32x4{0.f, 0.f, 0.f, 0.f};
    unsigned ev[4][2];
    f32x4 enk;
    f32x2 eig[2], efg[2], egg[2], eog[2], ecp[2], eex[2], etc[2], edc[2], eq[2];
    u32x4 elo, ehi;
    auto epi = [&](auto rpc, auto partc) {
      constexpr int RTp = decltype(rpc)::value, part = decltype(partc)::value, Kp = RTp % 4;
      constexpr int q = (part - 1) / 3, sub = (part - 1) % 3;
      if constexpr (part <= 6 && sub == 0) {
        const u32x4 sv = q == 0 ? sq0[Kp] : sq1[Kp];  // rows 2q, 2q+1: (i|f), (g|o) per row
        eig[q] = f32x2{__uint_as_float(sv[0] << 16), __uint_as_float(sv[2] << 16)};
        efg[q] = f32x2{__uint_as_float(sv[0] & 0xffff0000u), __uint_as_float(sv[2] & 0xffff0000u)};
        egg[q] = f32x2{__uint_as_float(sv[1] << 16), __uint_as_float(sv[3] << 16)};
        eog[q] = f32x2{__uint_as_float(sv[1] & 0xffff0000u), __uint_as_float(sv[3] & 0xffff0000u)};
        ecp[q] = f32x2{cval(Kp, 2 * q), cval(Kp, 2 * q + 1)};
        const f32x2 x2 = (efg[q] * ecp[q] + eig[q] * egg[q]) * 2.f;
        eex[q] = f32x2{__expf(x2[0]), __expf(x2[1])};
      } else if constexpr (part <= 6 && sub == 1) {
        etc[q] = 1.f - 2.f * f32x2{__builtin_amdgcn_rcpf(eex[q][0] + 1.f), __builtin_amdgcn_rcpf(eex[q][1] + 1.f)};
        const f32x2 dh = f32x2{dhp[2 * q], dhp[2 * q + 1]};
        const f32x2 kv = f32x2{dcr[RTp][2 * q], dcr[RTp][2 * q + 1]};
        eq[q] = dh * eog[q];
        edc[q] = eq[q] * (1.f - etc[q] * etc[q]) + kv;
        const f32x2 nk = edc[q] * efg[q];
        enk[2 * q] = nk[0];
        enk[2 * q + 1] = nk[1];
      } else if constexpr (part <= 6 && sub == 2) {
        const f32x2 a = edc[q] * eig[q], tq = a * egg[q];
        const f32x2 di = tq - tq * eig[q];          // dc g i (1 - i)
        const f32x2 dg = a - tq * egg[q];           // dc i (1 - g^2)
        const f32x2 u = edc[q] * efg[q] * ecp[q];
        const f32x2 df = u - u * efg[q];            // dc c_{t-1} f (1 - f)
        const f32x2 e = eq[q] * etc[q];
        const f32x2 dO = e - e * eog[q];            // dh tanh(c) o (1 - o)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          ev[2 * q + k][0] = pk_bf16(di[k], df[k]);  // one v_cvt_pk_bf16_f32 per pair
          ev[2 * q + k][1] = pk_bf16(dg[k], dO[k]);
        }
      } else if constexpr (part == 7) {
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
        if constexpr ((DBG & 4) != 0) {
          if (elo[0] == 0x7fc07fc1u && ehi[1] == 0x7fc07fc1u) dcr[RTp][0] = 1.f;  // keep the values live
        } else {
          constexpr int AUX = (DBG & 64) ? 0 : 16;  // sc1 (write-through) unless released
          __builtin_amdgcn_raw_buffer_store_b128(elo, dg_rsrc, st_base, SOFF, AUX);
          __builtin_amdgcn_raw_buffer_store_b128(ehi, dg_rsrc, st_base, SOFF + 2 * G * 2, AUX);
        }
      }
    };

    // The cell backward as 64 micro-stages in scalar fp32, one per MFMA of the next tile's loop
    // (at most two plain ops or one transcendental: what a 16x16x32 MFMA leaves free of its
    // 16 issue cycles; packed fp32 costs more issue beside MFMAs than two scalar ops).
    // Stage q < 60: rows 2p, 2p+1 (p = q / 30) in flight together, stage (q % 30) / 2 of row
    // 2p + (q & 1); q = 60: lane-pair exchange (part 7); q = 62: DG stores (part 8). Every
    // stage pins its values with empty "+v" asm, so the compiler can neither sink the math
    // below the MFMAs nor hoist it above them (it had gathered each part into one clump).
    // WELLFLOW_PF_DBG=512: the 8-part schedule instead (A/B).
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
    // exchanges at once (its cell backward drains before the hand-off).
    f32x4 dho = f32x4{0.f, 0.f, 0.f, 0.f};  // own partial of the previous tile (its unit tile)
    const unsigned rd_base = lds0 + RED + wid * 1024 + lane * 16;  // red[.][.][wid][lane]
    auto kt_of_part = [](int p) { return 2 * p - 1 + (p == 1 ? 1 : 0); };  // parts at k-tiles 2,3,5,..,15

    static_for<0, NRT>([&](auto rc) {
      constexpr int RT = decltype(rc)::value, P = RT & 1;
      // ---- wait for A(RT): its pieces were issued in the first half of tile RT-1's MFMA loop;
      // after the last one came tile RT-1's S / c loads (of tile RT+1 or of the next step) and
      // tile RT-2's DG stores (epilogue part 8, if RT-1 > 0), which may stay in flight
      if constexpr (RT == 0)
        wait_vmcnt<0>();
      else
        wait_vmcnt<NSC + (RT >= 2 ? NST : 0)>();
      stamp(s, 2 + 5 * RT);
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
      if constexpr (KT > 1 && (DBG & 4096) == 0)
        asm volatile("ds_read_b128 %0, %1" : "=v"(a[1]) : "v"(cur + fa[1]) : "memory");
      static_for<0, KT>([&](auto kc) {
        constexpr int kt = decltype(kc)::value;
        (void)acc;  // odr-use outside the asm operands: clang does not capture them implicitly
        (void)w;
        (void)pr;
        // A/B (WELLFLOW_PF_DBG=4096, production-correct): the round-2 one-ahead prefetch
        constexpr int AHEAD = (DBG & 4096) ? 1 : 2;
        if constexpr (kt + AHEAD < KT)
          asm volatile("ds_read_b128 %0, %1 offset:%2"
                       : "=v"(a[(kt + AHEAD) % 3])
                       : "v"(cur + fa[(kt + AHEAD) & 1]), "i"(((kt + AHEAD) >> 1) * 2048)
                       : "memory");
        // k-tile whose top sums the partials: 2, or 1 where the cell backward's first use of dh
        // (micro-stage 7) already falls into k-tile 1 (KT = 4, H = 128)
        constexpr int KSUM = (KT >= 8 && AHEAD == 2) ? 2 : 1;
        constexpr int YOUNGER = (kt + 1 < KT ? 1 : 0) + (AHEAD == 2 && kt + 2 < KT ? 1 : 0) +
                                (RT > 0 && kt == 1 && KSUM == 2 ? 3 : 0);
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(YOUNGER) : "memory");
        if constexpr (RT > 0 && kt == KSUM) {
          // the wait above drained the partial reads issued at k-tile 0 (LDS returns in order:
          // only the fragment reads after them are younger): tie them to it, then the previous tile's dh
          asm volatile("" : "+v"(pr[0]), "+v"(pr[1]), "+v"(pr[2]), "+v"(pr[3]));
          dhp = dho + ((pr[0] + pr[1]) + (pr[2] + pr[3]));
        }
        static_for<0, 4>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if constexpr (!(DBG & 2)) {
            if constexpr (kt == 0)
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc[j]) : "v"(a[kt % 3]), "a"(w[kt][j]));
            else
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(a[kt % 3]), "a"(w[kt][j]));
          }
          if constexpr (MICRO && RT > 0) {
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
        // last piece lands well before the next tile needs it
        if constexpr (RT + 1 < NRT && 2 * kt < KT) {
          issue_a(std::integral_constant<int, RT + 1>{}, std::integral_constant<int, 2 * kt>{});
          issue_a(std::integral_constant<int, RT + 1>{}, std::integral_constant<int, 2 * kt + 1>{});
        }
        if constexpr (kt == KT / 2 - 1) {  // S / c of tile RT + 2 right after the last A piece
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (RT + 2 < NRT)
            load_sc(t, std::integral_constant<int, RT + 2>{}, std::integral_constant<int, (RT + 2) % 4>{});
          else  // tiles 0 / 1 of the next step (t - 1; past step 0: a harmless reload, same count)
            load_sc(t > 0 ? t - 1 : t, std::integral_constant<int, RT + 2 - NRT>{},
                    std::integral_constant<int, (RT + 2) % 4>{});
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (RT > 0 && kt == 0) {
          // every wave's partial writes of tile RT-1 were drained by its lgkmcnt wait above
          __builtin_amdgcn_s_barrier();
          static_for<0, 4>([&](auto wc) {
            constexpr int w2 = decltype(wc)::value;
            (void)pr;
            (void)rd_base;
            if (w2 != wid)
              asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(pr[w2]) : "v"(rd_base),
                           "i"((((RT - 1) & 1) * 4 + w2) * 4 * 1024) : "memory");
            else
              pr[w2] = f32x4{0.f, 0.f, 0.f, 0.f};
          });
        }
        // parts of the previous tile's cell backward (part p at k-tile kt_of_part(p))
        static_for<1, EPI_PARTS + 1>([&](auto pc) {
          constexpr int p = decltype(pc)::value;
          if constexpr (!MICRO && RT > 0 && 2 * p - 1 + (p == 1 ? 1 : 0) == kt)
            epi(std::integral_constant<int, RT - 1>{}, pc);
        });
        // the MFMAs above are inline asm, so the compiler knows neither their latency nor that
        // they still read this fragment: keep its registers allocated until here, so no VALU
        // result of the interleaved epilogue can land in them while the MFMAs are in flight
        asm volatile("" ::"v"(a[kt % 3]));
      });
      (void)kt_of_part;
      // parts that did not fit a short loop
      static_for<1, EPI_PARTS + 1>([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        if constexpr (!MICRO && RT > 0 && 2 * p - 1 + (p == 1 ? 1 : 0) >= KT) epi(std::integral_constant<int, RT - 1>{}, pc);
      });
      // VALU / LDS reads of MFMA results: cover the pipeline (nothing is padded after asm)
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((DBG & 32) != 0) {  // MFMA completion: consume a result before stamping
        float sink = acc[3][3];
        asm volatile("" ::"v"(sink));
        stamp(s, 3 + 5 * RT);
      }

      // ---- K-split partials -> red[P] (the own unit tile stays in registers: dho)
      dho = wid == 0 ? acc[0] : wid == 1 ? acc[1] : wid == 2 ? acc[2] : acc[3];
      const unsigned rbase = lds0 + RED + (P * 4 + wid) * 4 * 1024 + lane * 16;  // red[P][wid][.][lane]
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j != wid) asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(rbase), "v"(acc[j]), "i"(j * 1024) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      stamp(s, 4 + 5 * RT);
      if constexpr (RT + 1 == NRT) {  // last tile: exchange now, drain its cell backward
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        static_for<0, 4>([&](auto wc) {
          constexpr int w2 = decltype(wc)::value;
          (void)acc;
          (void)rd_base;
          if (w2 != wid)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(acc[w2]) : "v"(rd_base), "i"((P * 4 + w2) * 4 * 1024) : "memory");
        });
        // the wait takes the accumulators as operands: the compiler sees inline-asm outputs as
        // ready at once and would otherwise schedule the sum between the reads and the wait
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]) :: "memory");
        dhp = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        stamp(s, 5 + 5 * RT);
        if constexpr (MICRO)
          static_for<0, 64>([&](auto qc) { bstage(std::integral_constant<int, RT>{}, qc); });
        else
          static_for<1, EPI_PARTS + 1>([&](auto pc) { epi(std::integral_constant<int, RT>{}, pc); });
      }
      stamp(s, 6 + 5 * RT);
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  // completion count (DONE vs EXPECT, persistent_guard.h)
  if (threadIdx.x == 0) pguard_done(stat, (unsigned)(d.T - 1));
}

template <int KT, int NRT>
static int launch_pb(const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S, bf16_t* DG, const float* dcarry,
                      unsigned* sync, unsigned* stat, int grid, LstmDims d, hipStream_t s) {
  const void* f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT>);
#ifdef WF_DIAG  // A/B and timing-only variants: diagnostic builds only (WELLFLOW_DIAG_BUILD=1)
  const void* const prod = f;
  if constexpr (KT == 16 && NRT == 16) {
    switch (d.dbg & 0xFFFFF) {
      case 4096: if constexpr (WF_DV(4096)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 4096>); break;  // 1-ahead DG ring
      case 1: if constexpr (WF_DV(1)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 1>); break;
      case 2: if constexpr (WF_DV(2)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 2>); break;
      case 4: if constexpr (WF_DV(4)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 4>); break;
      case 8: if constexpr (WF_DV(8)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 8>); break;
      case 16: if constexpr (WF_DV(16)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 16>); break;
      case 32: if constexpr (WF_DV(32)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 32>); break;
      case 64: if constexpr (WF_DV(64)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 64>); break;
      case 96: if constexpr (WF_DV(96)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 96>); break;
      case 128: if constexpr (WF_DV(128)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 128>); break;
      case 256: if constexpr (WF_DV(256)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 256>); break;
      case 512: if constexpr (WF_DV(512)) f = reinterpret_cast<const void*>(&lstm_bwd_persistent_kernel<KT, NRT, 512>); break;  // 8-part epilogue
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
