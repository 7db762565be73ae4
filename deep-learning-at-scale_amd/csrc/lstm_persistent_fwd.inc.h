// wellflow — persistent LSTM forward: ONE launch runs all T timesteps (kernel template; the
// instantiations are lstm_pf_parts.hip, the host launcher lstm_persistent.hip)
// (SURVEY.md §2.4 K13 "persistent kernel over T, W sliced across CUs, per-step agent-scope
// hand-off of h_t"; §7.4 hard part 2).
//
// Why: the per-step kernel (lstm.hip) re-streams its whole 256x256 weight tile from L2 /
// Infinity Cache every step (576 KB per CU per step with the activations) and pays a grid
// fill/drain per step. Here the weights never move after the prologue:
//  * grid = (B / (64*NC)) row blocks x (4H / 256) gate-column blocks, one 256-thread
//    workgroup (4 waves, one per SIMD) per CU, all co-resident (persistent_launch.h).
//  * wave w of column block n keeps Wp[gate cols n*256 + 64w .. +63][0:KA] — the four
//    gates of 16 hidden units (see the permutation in lstm.hip) — as MFMA B fragments in
//    registers for the whole sequence: KA/32 x 4 bf16x8 = 288 VGPRs at KA = 576.
//  * per step the workgroup streams its rows of [x_t | 1 | h_{t-1}] through a 2-deep LDS
//    ring of 64-row chunks (global_load_lds, 72 KB per chunk), so only activations move:
//    half the bytes of the per-step kernel.
//  * the fused cell epilogue is the per-step kernel's (same FN layouts for C / S, so the
//    backward pass is unchanged); h_t is staged through LDS and published with 8-B
//    write-through (sc1) stores.
//  * hand-off (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH.md "Valid forms" row 1):
//    h is stored sc1, every storing wave drains its stores before a workgroup barrier behind
//    which ONE lane adds to an arrival counter (agent-scope atomic), consumers poll it with sc1
//    loads and then load the chunk with sc1 LDS-DMA — no acquire. Counters only count up
//    (persistent_sync.h: launch epochs, no per-launch memset). At NC = 8 the hand-off is
//    SPLIT-PHASE per chunk (see SPLIT below): no step-top stop. Only the NB workgroups of one
//    row block depend on each other, so row blocks drift freely (no grid barrier), and the
//    XCD-aware block map puts a row block's NB workgroups on one XCD (speed only).
//  * every spin is bounded: a wave that times out records why and runs on without waiting
//    (results garbage, reported through the STAT block), so nothing can hang.
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
constexpr int PF_ROWS = 32;               // rows per ring chunk
constexpr unsigned PF_SPIN_LIMIT = 1u << 21;
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

// one cell element in flight through the forward's micro-staged epilogue
struct EpiMicro {
  float zi, zf, zg, zo, ei, ef, eg, eo, ig, fg, gg, og, cn, ec;
  unsigned p0, p1;
};
// empty volatile asm: the value must exist in a VGPR at this point of the instruction stream
// The value is redefined there ("+v"), so its consumers stay after this point too. (Input-
// only pins avoid the hazard recognizer's s_nop after every such asm, but let the compiler
// regroup the stages and shuffle values through AGPRs: 2.21 vs 1.50 ms per forward.)
__device__ __forceinline__ void pin(float& a) { asm volatile("" : "+v"(a)); }
template <typename A, typename B> __device__ __forceinline__ void pin(A& a, B& b) {
  asm volatile("" : "+v"(a), "+v"(b));
}
}  // namespace

// KT = KA / 32 k-tiles; NC = 32-row chunks per workgroup per step (compile-time, so every
// ring slot, LDS offset and vmcnt count below is an immediate).
template <int KT, int NC, int DBG = 0>  // DBG: timing-only builds (2 no MFMA, 4 no C/S stores, 8 no c loads; 64 stores in the loop)
__global__ __launch_bounds__(256, 1) void lstm_fwd_persistent_kernel(
    bf16_t* __restrict__ XH, const bf16_t* __restrict__ Wp, bf16_t* __restrict__ Cst,
    bf16_t* __restrict__ S, unsigned* __restrict__ sync, unsigned* __restrict__ stat, LstmDims d) {
  constexpr int KA = 32 * KT;
  constexpr int KS = KA / 64;                // 64-deep k-steps = A pieces per wave per chunk
  constexpr int ABYTES = PF_ROWS * KA * 2;   // chunk of [x_t | 1 | h_t-1] rows: KS [32][64] images
  constexpr int LPT = KS;                    // LDS-DMA instructions per wave per chunk
  // k-tiles whose weight fragments live in AGPRs (the rest in VGPRs): 256 AGPRs minus 2 x 32
  // accumulator registers (this chunk + the pipelined previous one) = 12 k-tiles x 4 x 4
  // KT = 20 (KX = 128, H = 512): 14 k-tiles in AGPRs (224 + the 32 accumulators = 256), so
  // the VGPR-resident weights stay at 6 k-tiles as at KT = 18
  constexpr int KTA_ = KT < 12 ? KT : (KT >= 20 ? 14 : 12);
  constexpr int NSTORE = (DBG & 4) ? 1 : 7;  // stores per wave per chunk: 2 C, 4 S, 1 h
  // one asm statement per MFMA + cell-math micro-stage (H = 512; WELLFLOW_PF_DBG=512: pinned
  // C++ micro-stages instead, for A/B)
  constexpr bool FUSED = KT >= 18 && (DBG & (2 | 128 | 512)) == 0;  // slots >= 144: plain MFMAs
  // the step top issues only chunk 0's pieces, so chunk 0 starts sooner after the hand-off
  // (every workgroup of the grid fetches its first chunks at once there); chunk 0 issues
  // chunks 1 and 2 from its MFMA loop (WELLFLOW_PF_DBG=1024: both at the step top, A/B)
  constexpr bool PF01 = NC >= 3 && (DBG & (2 | 1024)) == 0;
  // SPLIT-PHASE hand-off (round 5, NC = 8: the rows of ONE chunk depend only on the same
  // chunk of the previous step, whose h every workgroup of the row block publishes three
  // chunks after finishing it — round 6, was two: the publishing wait no longer covers the h
  // store just issued): one arrival counter per chunk, the chunk pieces two chunks ahead
  // across the step boundary (chunks 0 / 1 of step t+1 during chunks NC-2 / NC-1 of step t),
  // the last chunk's cell epilogue in the next step's first MFMA loop like any other, and a
  // per-wave sc1 poll one chunk before each fetch — no step-top stop. A 4-slot ring (slot =
  // chunk % 4 in every step). Smaller NC keep the per-step hand-off: a chunk's own next-step
  // input would be published too late to fetch ahead (NC < 8), or at all (NC = 1).
  constexpr bool SPLIT = NC == 8 && 4 * ABYTES + PF_ROWS * 64 * 2 + 32 <= 163840;  // KX = 128: 3 slots only
  constexpr int NSLOT = SPLIT ? 4 : 3;
  // ALT (DBG 2048, A/B only; measured SLOWER: 1.36 vs 1.28 ms interleaved,
  // profiles/r6/forward_budget.md): the accumulators in VGPRs as TWO sets that alternate
  // between chunk bodies (body P accumulates into set P & 1 while its fused cell stages read the
  // previous chunk's set directly), so no chunk copies its 32 accumulators out of the AGPRs and
  // 14 k-tiles of weights fit the AGPR file. Production keeps the AGPR accumulators + copy.
  constexpr bool ALT = FUSED && SPLIT && (DBG & 2048) != 0;
  // SPLIT publish delay (round 6): chunk j publishes chunk j - PD, polled one chunk before its
  // fetch; DBG 262144 (A/B): the round-5 form, PD = 2 with the poll two chunks before
  constexpr bool PUB3 = (DBG & 262144) == 0;
  // PL: the poll read at a chunk top was issued PL chunks earlier. PL = 2 (production): the
  // top of chunk j no longer waits for chunk j+1's pieces (issued just before the poll of
  // j-1): 1.30 vs 1.38 ms interleaved, all 8 paired windows faster (profiles/r6/diag/ab2.txt)
  // although the staler polls block more often (294 vs 191 waits per launch).
  // DBG 8 (A/B): PL = 1, the first round-6 form
  constexpr int PD = PUB3 ? 3 : 2, PL = (PUB3 && (DBG & 8) != 0) ? 1 : 2;
  // DBG 256 (A/B, measured slower): each wave publishes its own 32-B piece of every h row
  // (no staging barrier); the production form writes whole 128-B lines, one per 8 lanes
  constexpr bool WAVE_H = (DBG & 256) != 0;
  constexpr bool NOHO = (DBG & 524288) != 0;  // timing only: no hand-off (no publish, poll or wait)
  constexpr int KTA = ALT ? 14 : KTA_;
  // Distinct static LDS objects per ring slot: the compiler then proves the slot being
  // filled by LDS-DMA disjoint from the slots being read, and inserts no vmcnt(0) of its own.
  // EXACTLY ONE static LDS variable, compile-time offsets for every ring slot, the h staging
  // area and the flag word (slot k at k*SLOT: one A chunk). With several LDS
  // variables the LDS lowering gives each its own alias scope, the waitcnt pass then tracks
  // the LDS-DMA into the ring and guards the first read of every slot with vmcnt(0) — which
  // drained the whole prefetch ring every chunk (measured: loads no longer overlapped MFMA).
  constexpr int SLOT = ABYTES;
  constexpr int HOFF = NSLOT * SLOT, FOFF = HOFF + PF_ROWS * 64 * 2;
  // [FOFF] flag, [FOFF + 8] epoch | ordinal, [FOFF + 16] per-wave failed words
  __shared__ __attribute__((aligned(16))) char smem[FOFF + 32];
  // h_t staging [32][64] bf16, accessed only through inline asm (32-bit LDS address)
  const unsigned hb_lds = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)(smem + HOFF));
  const unsigned flag_lds = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)(smem + FOFF));
  const unsigned lds_smem = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);

  // KX (x block + bias column, padded) = 64 for F <= 63, 128 for F <= 127; KT = KA / 32 tells
  // them apart for H in {128, 256, 512}: 6 / 10 / 18 at KX = 64, 8 / 12 / 20 at KX = 128
  constexpr int KXC = (KT == 8 || KT == 12 || KT == 20) ? 128 : 64;
  constexpr int H = KA - KXC, G = 4 * H, NB = G / 256, HB = H / 16;
  static_assert(H == 128 || H == 256 || H == 512, "KT must encode (KX, H)");
  const int Bp = fn_rows(d.B);
  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int m = L / NB, n = L % NB;
  const int row0 = m * PF_ROWS * NC + d.row_off;  // row_off: sub-batch origin (launcher)
  const int ub = n * 4 + wid;                // 16-unit block of this wave
  const int u = ub * 16 + l15;               // hidden unit of this lane
  const int loff_c = ub * 256 + lane * 4;    // element offset of this lane's C slot (4 bf16) in a FN row block
  // bf16 offset of this lane's first S half in a FN row block (DBG 32768, timing only: the round-2
  // lane-interleaved 32-B slot, second half 16 B after the first)
  constexpr int SHALF = (DBG & 32768) ? 8 : kFnSHalf;
  const int loff_s = ub * 1024 + lane * ((DBG & 32768) ? 16 : 8);
  const int loff_h = (((int)threadIdx.x >> 3) * KA + ((int)threadIdx.x & 7) * 8) * 2;  // h publish
  // SPLIT: each wave publishes its OWN 16 units of the chunk's 32 rows (row lane >> 1, 8-unit
  // half lane & 1: 32 B per row per wave), so its LDS staging needs no workgroup barrier
  const int loff_hw = ((lane >> 1) * KA + wid * 16 + 8 * (lane & 1)) * 2;
  const unsigned hb_rd = hb_lds + (unsigned)((lane >> 1) * 128 + wid * 32 + (lane & 1) * 16);
  // error word: word 0 of the per-launch block (word 1 in the round-2 layout A/B, PF_DBG bit 20)
  // production objects keep only the test hook bit (kDbgMask, persistent_guard.h): the
  // timing-only branches below fold away at compile time
  const int dbg = d.dbg & kDbgMask;
  ps_u32* rbw = psync_rb(sync, m);
  ps_u32* err = rbw + kPSyncErr;
  const unsigned spin_limit = d.spin_limit ? d.spin_limit : PF_SPIN_LIMIT;
  // (dbg bit 21, tests: an unreachable target, so the polls fail and the bounded spin trips)
  const unsigned force = ((dbg >> 21) & 1u) << 30;
  // DBG & 16: timeline stamps (s_memrealtime, 100 MHz) of step PF_STAMP_T, wave 0 lane 0 of
  // every workgroup, into sync + 4096 words (64 slots per workgroup; diagnostics only)
  constexpr int PF_STAMP_T = 10;
  unsigned long long* stamps = reinterpret_cast<unsigned long long*>(sync + 4096) + blockIdx.x * 64;
  auto stamp = [&](int t, int slot) {
    if constexpr ((DBG & 16) != 0) {
      if (t == PF_STAMP_T && threadIdx.x == 0) stamps[slot] = __builtin_amdgcn_s_memrealtime();
    }
  };

  // completion guard (persistent_guard.h) and this launch's epoch (persistent_sync.h)
  if (threadIdx.x == 0) {
    const unsigned o = pguard_start(stat, (unsigned)d.T);
    // a buffer last used by a launch of another (NC, T, NB) fails loudly (persistent_sync.h)
    const unsigned sig = psync_sig(0u, (unsigned)NC, (unsigned)d.T, (unsigned)NB);
    const unsigned bad = psync_check_sig(sync, sig);
    if (bad) {
      pguard_exit(stat, 0u, 5u, bad, 0u, sig, 0u, o);
      pguard_sticky(stat);
    }
    const unsigned e = __hip_atomic_fetch_add(rbw + kPSyncStart, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) / NB;
    asm volatile("ds_write_b64 %0, %1" ::"v"(flag_lds + 8), "v"((unsigned long long)e | ((unsigned long long)o << 32))
                 : "memory");
    asm volatile("ds_write_b32 %0, %1" ::"v"(flag_lds), "v"(bad) : "memory");
  }
  // ---- prologue: stationary weight fragments (B operand: lane holds col l15, k 8g..8g+7)
  bf16x8 w[KT][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16_t* wr = Wp + (size_t)(n * 256 + wid * 64 + j * 16 + l15) * KA + 8 * g;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) w[kt][j] = *reinterpret_cast<const bf16x8*>(wr + 32 * kt);
  }
  // drain them with a wait the compiler's counter model sees (the memory clobber keeps the
  // loads above it), so it does not re-wait for them at the top of every step
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  unsigned long long eo;
  unsigned sigbad;
  asm volatile("ds_read_b64 %0, %2\n\tds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(eo), "=&v"(sigbad)
               : "v"(flag_lds + 8), "v"(flag_lds)
               : "memory");
  const unsigned epoch = __builtin_amdgcn_readfirstlane((unsigned)eo);
  const unsigned ord = __builtin_amdgcn_readfirstlane((unsigned)(eo >> 32));
  const unsigned tag = epoch + 1u;
  // arrivals a consumer needs before step tt reads chunk cc (SPLIT) / before step tt (per-step
  // hand-off): every workgroup of the row block published it for steps 0 .. tt-1. SPLIT
  // publishes chunk cc at the top of chunk cc + 3: in every step for cc <= NC-4, in all but the
  // last step for the last three chunks; the per-step hand-off counts steps 1 .. T-1.
  auto target = [&](int cc, int tt) -> unsigned {
    const unsigned per_launch = SPLIT ? (unsigned)(cc <= NC - 1 - PD ? d.T : d.T - 1) : (unsigned)(d.T - 1);
    return epoch * (unsigned)NB * per_launch + (unsigned)(NB * (SPLIT ? tt : tt)) + force;
  };
  // uniform: this wave failed a hand-off or the signature check (runs on, never waits again)
  unsigned failed = __builtin_amdgcn_readfirstlane(sigbad) != 0u ? 1u : 0u;
  // SPLIT: blocking wait of this wave for chunk cc before step tt reads it (a poll that did
  // not match); a failure is recorded once and makes every later wait a no-op
  auto wait_chunk = [&](int cc, int tt) {
    if (failed) return;
#ifdef WF_DIAG
    if (lane == 0) pguard_add(stat + 20, 1u);  // diagnostics: blocking waits (tools/pf_budget.py)
#endif
    unsigned seen_cnt = 0, seen_err = 0;
    const unsigned tg = target(cc, tt);
    const unsigned why = psync_wait(rbw + kPSyncGroup + cc, err, tg, tag, spin_limit, stat, &seen_cnt, &seen_err);
    if (why != 0) {
      failed = 1;
      if (lane == 0) pguard_exit(stat, (unsigned)tt, why, seen_err, seen_cnt, tg, (unsigned)cc, ord);
    }
  };
  // sc1 poll of chunk cc's counter (one uniform load; inline asm, so it stays where written
  // and the chunk-top wait that covers it names its register)
  auto poll = [&](int cc) {
    unsigned v;
    const unsigned* pa = sync + kPSyncHead + kPSyncRowBlock * m + kPSyncGroup + cc;
    asm volatile("global_load_dword %0, %1, off sc1" : "=v"(v) : "v"(pa) : "memory");
    return v;
  };
  unsigned pvr[2] = {0u, 0u};  // SPLIT: the polls in flight (chunk j polls for chunk j + 2 + PL)
  // per-step store bases of the previous step (SPLIT: chunk 0 finalizes the previous step's
  // last chunk)
  bf16_t* cnext_p = nullptr;
  bf16_t* St_p = nullptr;
  __amdgpu_buffer_rsrc_t xh_rsrc_p = __builtin_amdgcn_make_buffer_rsrc(XH, 0, 0, 0x00020000);

  // A piece s of this wave: k-step s, rows wid*8 + (lane>>3); the K_CONTIG 16-B chunk
  // swizzle (row>>1)&7 = 4(wid&1) + g is lane-constant, so it moves onto the source offset.
  const unsigned aoff = (unsigned)((wid * 8 + (lane >> 3)) * KA * 2 + (((lane & 7) ^ (4 * (wid & 1) + g)) << 4));
  int fa[2];  // A fragment offsets in a [32][64] image (rows l15 of a 16-row tile)
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) fa[kk] = l15 * 128 + (((kk * 4 + g) ^ ((l15 >> 1) & 7)) << 4);

  // c_{t-1} of the workgroup's 8 chunks stays in registers for the whole sequence (a queue
  // the chunk loop rotates: chunk c reads cq[0] and appends its c_t), so the forward never
  // re-reads the cell state it wrote (16.8 MB per step at B = 8192); C is still stored for
  // the backward. c_{-1} = 0.
  f32x4 cq[NC][2];
#pragma unroll
  for (int q = 0; q < NC; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i) cq[q][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 accp[2][4];  // gate pre-activations of the previous chunk (software pipeline; !ALT)
  f32x4 accs[2][2][4];  // ALT: the two alternating accumulator sets
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) accs[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) accp[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int t = 0; t < d.T; ++t) {
    stamp(t, 0);
    if (!SPLIT && t > 0) {
      // ---- per-step hand-off (NC < 8): publish step t-1 (every wave drained its sc1 h
      // stores: issued before the drain's NSTORE - 1 C / S stores, which may stay in flight),
      // then thread 0 waits for the row block; the other waves load after the barrier it
      // joins (MI355X_MICROARCH.md "Valid forms" row 1: sc1 stores, sc1 loads, no acquire)
      wait_vmcnt<NSTORE - 1>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      stamp(t, 62);  // h stores drained, workgroup arrived
      if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(rbw + kPSyncGroup, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned f = failed;
        if (!f) {
          unsigned seen_cnt = 0, seen_err = 0;
          const unsigned tg = target(0, t);
          const unsigned why = psync_wait(rbw + kPSyncGroup, err, tg, tag, spin_limit, stat, &seen_cnt, &seen_err);
          if (why != 0) {
            f = 1;
            pguard_exit(stat, (unsigned)t, why, seen_err, seen_cnt, tg, 0u, ord);
          }
        }
        stamp(t, 63);  // row block complete (poll matched)
        asm volatile("ds_write_b32 %0, %1" ::"v"(flag_lds), "v"(f) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // the flag word through ds_read in asm (a volatile C++ access became a flat load with
      // sc0 sc1 and a vmcnt + lgkmcnt wait, every step)
      unsigned fv;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(fv) : "v"(flag_lds) : "memory");
      failed = __builtin_amdgcn_readfirstlane(fv);  // a failed workgroup runs on without waiting
    }
    stamp(t, 1);
    // opaque per-step copy of the row origin: stops the compiler hoisting every chunk's
    // lane addresses out of the time loop (NC x 64-bit offsets live across the whole
    // kernel pushed the H = 512, NC = 8 build into spills)
    int rb = row0;
    asm volatile("" : "+s"(rb));
    // per-step uniform bases (row block origin folded in) + per-lane constant offsets
    // (loff_c / loff_s / loff_h), so every chunk address is base + compile-time stride
    // c_t history for the backward, bf16 (the forward itself carries c in fp32 registers, cq)
    bf16_t* cnext = Cst + (size_t)(t + 1) * Bp * H + (size_t)(rb >> 4) * HB * 256;
    bf16_t* St = S + (size_t)t * Bp * G + (size_t)(rb >> 4) * HB * 1024;
    const char* abase = reinterpret_cast<const char*>(XH + ((size_t)t * d.B + rb) * KA) + aoff;
    // SPLIT: the next step's A (XH has T + 1 slabs, so slab t + 1 always exists)
    const char* abase_n = reinterpret_cast<const char*>(XH + ((size_t)(t + 1) * d.B + rb) * KA) + aoff;
    // slab t + 1 of XH as a buffer resource for the 16-B sc1 h stores: per-slab byte offsets
    // (< B * KA * 2 < 2^31, host-checked) so any batch size fits the 32-bit offsets
    const __amdgpu_buffer_rsrc_t xh_rsrc =
        __builtin_amdgcn_make_buffer_rsrc(XH + (size_t)(t + 1) * d.B * KA, 0, 0x7FFFFFFF, 0x00020000);
    const int hsoff = (int)(((size_t)rb * KA + KXC + n * 64) * 2);

    // cell epilogue element (row-tile i, row r) of the carried chunk: accp + c_{t-1} = cq[0]
    auto epi_elem_src = [&](const f32x4 (&src)[2][4], int i, int r, float (&cv)[2][4], unsigned (&pk)[2][8],
                            unsigned (&hv)[2][4]) {
      const float ig = sigmoid_pre(src[i][0][r]);  // Wp carries the gate scales (pack kernel)
      const float fg = sigmoid_pre(src[i][1][r]);
      const float gg = tanh_pre(src[i][2][r]);
      const float og = sigmoid_pre(src[i][3][r]);
      const float cn = fg * cq[0][i][r] + ig * gg;
      cv[i][r] = cn;
      pk[i][2 * r] = pk_bf16(ig, fg);
      pk[i][2 * r + 1] = pk_bf16(gg, og);
      hv[i][r] = f2bf(og * tanhf_(cn));
    };
    auto epi_elem = [&](int i, int r, float (&cv)[2][4], unsigned (&pk)[2][8], unsigned (&hv)[2][4]) {
      if constexpr (ALT)
        epi_elem_src(accs[(NC - 1) & 1], i, r, cv, pk, hv);  // the drain: the last chunk's set
      else
        epi_elem_src(accp, i, r, cv, pk, hv);
    };
    // The same element in two halves pinned to k-tile positions of the next chunk's MFMA
    // loop. Empty asm statements take the inputs and produce the outputs at that point:
    // the MFMAs are volatile asm too, so the compiler can neither hoist the cell math above
    // the loop nor sink it below (it sank all of it: 144 MFMAs back to back, then ~280 VALU
    // with the matrix core idle). Half 0: i, f, g gates and c_t; half 1: o gate, tanh(c_t),
    // h_t and the packed gate words.
    auto epi_half = [&](int hh, int i, int r, float (&cv)[2][4], float (&gs)[2][4], unsigned (&pk)[2][8],
                        unsigned (&hv)[2][4]) {
      if (hh == 0) {
        float zi = accp[i][0][r], zf = accp[i][1][r], zg = accp[i][2][r], cp = cq[0][i][r];
        asm volatile("" : "+v"(zi), "+v"(zf), "+v"(zg), "+v"(cp));
        const float ig = sigmoid_pre(zi), fg = sigmoid_pre(zf), gg = tanh_pre(zg);
        float cn = fg * cp + ig * gg;
        unsigned p0 = pk_bf16(ig, fg);
        float g2 = gg;
        asm volatile("" : "+v"(cn), "+v"(p0), "+v"(g2));
        cv[i][r] = cn;
        pk[i][2 * r] = p0;
        gs[i][r] = g2;
      } else {
        float zo = accp[i][3][r];
        asm volatile("" : "+v"(zo));
        const float og = sigmoid_pre(zo);
        unsigned p1 = pk_bf16(gs[i][r], og);
        unsigned h = f2bf(og * tanhf_(cv[i][r]));
        asm volatile("" : "+v"(p1), "+v"(h));
        pk[i][2 * r + 1] = p1;
        hv[i][r] = h;
      }
    };
    // The element as 18 micro-stages, each at most one issue slot's worth of VALU (one
    // transcendental or two plain ops, <= 8 cycles: what a 16x16x32 MFMA leaves free of its
    // 16), placed one per MFMA of the next chunk's loop (8 x 18 = 144 = the MFMA count at
    // H = 512). Every stage pins its inputs and outputs with empty volatile asm, so it
    // stays between its two MFMAs.
    auto epi_micro = [&](auto sc, int i, int r, EpiMicro& e, float (&cv)[2][4], unsigned (&pk)[2][8],
                         unsigned (&hv)[2][4]) {
      constexpr int s = decltype(sc)::value;
      if constexpr (s == 0) {
        e.zi = accp[i][0][r];
        e.zf = accp[i][1][r];
        e.zg = accp[i][2][r];
        e.zo = accp[i][3][r];
        pin(e.zi, e.zf);
        pin(e.zg, e.zo);
      } else if constexpr (s == 1) {
        pin(e.zi); e.ei = __builtin_amdgcn_exp2f(e.zi); pin(e.ei);
      } else if constexpr (s == 2) {
        pin(e.zf); e.ef = __builtin_amdgcn_exp2f(e.zf); pin(e.ef);
      } else if constexpr (s == 3) {
        pin(e.zg); e.eg = __builtin_amdgcn_exp2f(e.zg); pin(e.eg);
      } else if constexpr (s == 4) {
        pin(e.zo); e.eo = __builtin_amdgcn_exp2f(e.zo); pin(e.eo);
      } else if constexpr (s == 5) {
        pin(e.ei, e.ef); e.ei += 1.0f; e.ef += 1.0f; pin(e.ei, e.ef);
      } else if constexpr (s == 6) {
        pin(e.ei); e.ig = __builtin_amdgcn_rcpf(e.ei); pin(e.ig);
      } else if constexpr (s == 7) {
        pin(e.ef); e.fg = __builtin_amdgcn_rcpf(e.ef); pin(e.fg);
      } else if constexpr (s == 8) {
        pin(e.eg, e.eo); e.eg += 1.0f; e.eo += 1.0f; pin(e.eg, e.eo);
      } else if constexpr (s == 9) {
        pin(e.eg); e.gg = __builtin_amdgcn_rcpf(e.eg); pin(e.gg);
      } else if constexpr (s == 10) {
        pin(e.eo); e.og = __builtin_amdgcn_rcpf(e.eo); pin(e.og);
      } else if constexpr (s == 11) {
        // c_t = fma(f, c_{t-1}, i * g): the contraction the per-step kernel's
        // f * c + i * g compiles to, so both paths round alike
        pin(e.gg, e.ig); e.gg = 1.0f - 2.0f * e.gg; e.cn = e.ig * e.gg; pin(e.gg, e.cn);
      } else if constexpr (s == 12) {
        pin(e.cn, e.fg); e.cn = __builtin_fmaf(e.fg, cq[0][i][r], e.cn); e.p0 = pk_bf16(e.ig, e.fg); pin(e.cn, e.p0);
      } else if constexpr (s == 13) {
        pin(e.og); e.p1 = pk_bf16(e.gg, e.og); e.ec = e.cn * 2.8853900817779268f; pin(e.p1, e.ec);
      } else if constexpr (s == 14) {
        pin(e.ec); e.ec = __builtin_amdgcn_exp2f(e.ec); pin(e.ec);
      } else if constexpr (s == 15) {
        pin(e.ec); e.ec = __builtin_amdgcn_rcpf(e.ec + 1.0f); pin(e.ec);
      } else if constexpr (s == 16) {
        pin(e.ec); e.ec = e.og * (1.0f - 2.0f * e.ec); pin(e.ec);
      } else {
        pin(e.ec);
        unsigned h = f2bf(e.ec);
        pin(h, e.cn);
        cv[i][r] = e.cn;
        pk[i][2 * r] = e.p0;
        pk[i][2 * r + 1] = e.p1;
        hv[i][r] = h;
      }
    };
    // The same three pieces, issued one by one from inside the next chunk's MFMA loop
    // (diagnostic build WELLFLOW_PF_DBG=64, KT >= 16): h staging, then one C / S store per
    // k-tile (issue order unchanged, so the vmcnt counts below still hold). Measured 1.64 vs
    // 1.60 ms for the stores after the loop (tools/pf_time.py 0,64): not the default.
    auto epi_h = [&](const unsigned (&hv)[2][4]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          asm volatile("ds_write_b16 %0, %1" ::"v"(hb_lds + 2u * ((i * 16 + 4 * g + r) * 64 + wid * 16 + l15)),
                       "v"(hv[i][r])
                       : "memory");
    };
    auto epi_cs = [&](int e, int k, const float (&cv)[2][4], const unsigned (&pk)[2][8]) {  // k = 0..5
      if constexpr (!(DBG & 4)) {
        const int i = k < 2 ? k : (k - 2) >> 1;
        if (k < 2) {
          *reinterpret_cast<uint2*>(cnext + (2 * e + i) * HB * 256 + loff_c) =
              make_uint2(pk_bf16(cv[i][0], cv[i][1]), pk_bf16(cv[i][2], cv[i][3]));
        } else {
          const int hf = (k - 2) & 1;
          uint4* sp = reinterpret_cast<uint4*>(St + (2 * e + i) * HB * 1024 + loff_s + hf * SHALF);
          *sp = make_uint4(pk[i][4 * hf], pk[i][4 * hf + 1], pk[i][4 * hf + 2], pk[i][4 * hf + 3]);
        }
      }
    };
    auto rotate = [&](const float (&cv)[2][4]) {
#pragma unroll
      for (int q = 0; q + 1 < NC; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i) cq[q][i] = cq[q + 1][i];
#pragma unroll
      for (int i = 0; i < 2; ++i) cq[NC - 1][i] = f32x4{cv[i][0], cv[i][1], cv[i][2], cv[i][3]};
    };
    // stores of chunk e (C, S: NSTORE - 1 per wave), h staged in LDS, c-queue rotation
    auto epi_store = [&](int e, const float (&cv)[2][4], const unsigned (&pk)[2][8], const unsigned (&hv)[2][4]) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          // LDS staging writes in asm: compiler-visible LDS writes are guarded by a vmcnt(0)
          // (the waitcnt pass orders every LDS access after in-flight LDS-DMA)
          asm volatile("ds_write_b16 %0, %1" ::"v"(hb_lds + 2u * ((i * 16 + 4 * g + r) * 64 + wid * 16 + l15)),
                       "v"(hv[i][r])
                       : "memory");
        if constexpr (!(DBG & 4)) {
          *reinterpret_cast<uint2*>(cnext + (2 * e + i) * HB * 256 + loff_c) =
              make_uint2(pk_bf16(cv[i][0], cv[i][1]), pk_bf16(cv[i][2], cv[i][3]));
          bf16_t* sb = St + (2 * e + i) * HB * 1024 + loff_s;
          *reinterpret_cast<uint4*>(sb) = make_uint4(pk[i][0], pk[i][1], pk[i][2], pk[i][3]);
          *reinterpret_cast<uint4*>(sb + SHALF) = make_uint4(pk[i][4], pk[i][5], pk[i][6], pk[i][7]);
        }
      }
#pragma unroll
      for (int q = 0; q + 1 < NC; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i) cq[q][i] = cq[q + 1][i];
#pragma unroll
      for (int i = 0; i < 2; ++i) cq[NC - 1][i] = f32x4{cv[i][0], cv[i][1], cv[i][2], cv[i][3]};
    };
    // publish chunk e's h rows: 32 rows x 128 B, one 16-B write-through (sc1) buffer store per
    // thread (Guideline 16 R1: no release fence; 8-B sc1 stores cost 0.4 ms more, measured)
    auto publish = [&](int e) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      u32x4 vv;  // row threadIdx>>3, 16-B column threadIdx&7 of the [32][64] bf16 tile
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(vv)
                   : "v"(hb_lds + 16u * threadIdx.x)
                   : "memory");
      __builtin_amdgcn_raw_buffer_store_b128(vv, xh_rsrc, loff_h, hsoff + e * PF_ROWS * KA * 2, 16 /* sc1 */);
    };

    // SPLIT: stores of chunk e with explicit bases (chunk 0 finalizes the previous step's last
    // chunk): h staged in LDS and stored FIRST (one 16-B sc1 store per thread), then the C / S
    // stores, so the next chunk top's vmcnt(NSTORE - 1) leaves only those in flight and the
    // chunk can be published there; then the c-queue rotation
    auto epi_store_split = [&](int e, bf16_t* cnx, bf16_t* stp, const __amdgpu_buffer_rsrc_t& xrs,
                               const float (&cv)[2][4], const unsigned (&pk)[2][8], const unsigned (&hv)[2][4]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          asm volatile("ds_write_b16 %0, %1" ::"v"(hb_lds + 2u * ((i * 16 + 4 * g + r) * 64 + wid * 16 + l15)),
                       "v"(hv[i][r])
                       : "memory");
      u32x4 vv;
      if constexpr (WAVE_H) {
        // the wave's own [32 rows][16 units] block back as 16-B pieces (LDS executes one wave's
        // accesses in order: no barrier). Measured +0.4 ms per forward: every 128-B h line is
        // then four 32-B write-through pieces from four waves instead of one whole-line store
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(vv) : "v"(hb_rd) : "memory");
        __builtin_amdgcn_raw_buffer_store_b128(vv, xrs, loff_hw, hsoff + e * PF_ROWS * KA * 2, 16 /* sc1 */);
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // row threadIdx>>3, 16-B column threadIdx&7 of the [32][64] bf16 tile: whole 128-B lines
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(vv) : "v"(hb_lds + 16u * threadIdx.x)
                     : "memory");
        __builtin_amdgcn_raw_buffer_store_b128(vv, xrs, loff_h, hsoff + e * PF_ROWS * KA * 2, 16 /* sc1 */);
      }
      if constexpr (!(DBG & 4)) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          *reinterpret_cast<uint2*>(cnx + (2 * e + i) * HB * 256 + loff_c) =
              make_uint2(pk_bf16(cv[i][0], cv[i][1]), pk_bf16(cv[i][2], cv[i][3]));
          bf16_t* sb = stp + (2 * e + i) * HB * 1024 + loff_s;
          *reinterpret_cast<uint4*>(sb) = make_uint4(pk[i][0], pk[i][1], pk[i][2], pk[i][3]);
          *reinterpret_cast<uint4*>(sb + SHALF) = make_uint4(pk[i][4], pk[i][5], pk[i][6], pk[i][7]);
        }
      }
      rotate(cv);
    };

    // chunk c -> ring slot c % 3: KS A pieces + this wave's 2 FN blocks of c_{t-1}
    auto issue = [&](int c, auto sc) {  // chunk c into ring slot SL (= c % 3)
      constexpr int SL = decltype(sc)::value;
      char* ra = smem + SL * SLOT;
      const char* src = abase + (size_t)c * ABYTES;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        __builtin_amdgcn_global_load_lds((const void*)(src + s * 128), (lds_void*)(ra + s * 4096 + wid * 1024),
                                         16, 0, 16 /* sc1 */);
    };
    // SPLIT: chunk c of the step whose A base is `base` into ring slot SL
    auto issue_b = [&](const char* base, int c, auto sc) {
      constexpr int SL = decltype(sc)::value;
      if constexpr ((DBG & 131072) != 0) return;  // timing only: no LDS-DMA after step 0 (stale A)
      char* ra = smem + SL * SLOT;
      const char* src = base + (size_t)c * ABYTES;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        __builtin_amdgcn_global_load_lds((const void*)(src + s * 128), (lds_void*)(ra + s * 4096 + wid * 1024),
                                         16, 0, 16 /* sc1 */);
    };
    auto issue_b0 = [&](const char* base, int c, auto sc) {  // step 0's first two chunks (every build)
      constexpr int SL = decltype(sc)::value;
      char* ra = smem + SL * SLOT;
      const char* src = base + (size_t)c * ABYTES;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        __builtin_amdgcn_global_load_lds((const void*)(src + s * 128), (lds_void*)(ra + s * 4096 + wid * 1024),
                                         16, 0, 16 /* sc1 */);
    };
    // piece s of chunk c into ring slot SL
    auto issue_piece = [&](int c, auto sc, int s) {
      constexpr int SL = decltype(sc)::value;
      const char* src = abase + (size_t)c * ABYTES;
      __builtin_amdgcn_global_load_lds((const void*)(src + s * 128), (lds_void*)(smem + SL * SLOT + s * 4096 + wid * 1024),
                                       16, 0, 16 /* sc1 */);
    };
    if constexpr (!SPLIT) {  // per-step hand-off: chunk 0 (and 1) at the step top
      issue(0, std::integral_constant<int, 0>{});
      if constexpr (NC > 1 && !PF01) issue(1, std::integral_constant<int, 1>{});
    }

    // chunk body, ring slot P = c % 3 compile-time (3 bodies in a runtime loop keep the
    // register pressure of a 3-chunk kernel; a fully unrolled NC = 8 spilled)
    // FIRST: chunk 0 with PF01 (compile-time c = 0): only its own pieces were issued at the
    // step top, and it issues chunks 1 and 2 one piece per k-tile from inside its MFMA loop
    auto chunk = [&](int c, auto pc, auto fc) {
      constexpr int P = decltype(pc)::value;
      constexpr bool FIRST = decltype(fc)::value;
      stamp(t, 2 + 5 * c);
      // vector-memory ops issued after chunk c's LDS-DMA (top of c issues c+2, then stores)
      // (issue order: prologue glds 0, 1; chunk k: glds k+2, then the stores of chunk k-1,
      // NSTORE per wave, none in chunk 0)
      // SPLIT: chunk j (global) waits until only chunk j-1's h and C / S stores are in flight:
      // its own pieces, chunk j+1's, the poll issued at the top of chunk j-1 (its register is
      // an operand: no use moves above the wait) and chunk j-3's h store (published below).
      // Round 6: the h store of chunk j-2, issued just before this wait, no longer has to land
      // first (it is published one chunk later), so no chunk top waits out a write-through.
      if constexpr (SPLIT) {
        if (t == 0 && c < 2)
          wait_vmcnt<LPT>();
        else
          // in flight at this wait (issue order): ... | top j-2: pieces j, poll | end j-2: h j-3, C/S
          // | top j-1: pieces j+1, poll | end j-1: h j-2, C/S (NSTORE - 1) | — PD = 3 keeps h j-2 in
          // flight (NSTORE), with PL = 2 also the pieces and poll of j-1 (the poll read here is j-2's)
          asm volatile("s_waitcnt vmcnt(%1)" : "+v"(pvr[P % PL])
                       : "n"(PD == 2 ? NSTORE - 1 : (PL == 1 ? NSTORE : NSTORE + LPT + 1)) : "memory");
      } else if (c == 0) {
        if (NC > 1 && !FIRST) wait_vmcnt<LPT>(); else wait_vmcnt<0>();
      } else if (c == 1) {
        if (NC > 2) wait_vmcnt<LPT>(); else wait_vmcnt<0>();
      } else if (c == 2) {
        if (NC > 3) wait_vmcnt<LPT + NSTORE>(); else wait_vmcnt<NSTORE>();
      } else if (c + 1 < NC) {
        wait_vmcnt<2 * NSTORE + LPT>();
      } else {
        wait_vmcnt<2 * NSTORE>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);  // keep each chunk's code (and live ranges) to itself
      stamp(t, 3 + 5 * c);
      if constexpr (SPLIT) {
        // publish chunk j-PD: every wave drained its h store before the barrier above
        if (!NOHO && (t > 0 || c >= PD) && threadIdx.x == 0)
          __hip_atomic_fetch_add(rbw + kPSyncGroup + (c >= PD ? c - PD : c + NC - PD), 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        // chunk j+2: its h rows were published by the row block 3 chunks ago; the poll of one
        // chunk ago says whether all arrived, else wait here (bounded)
        const int c2 = c + 2 < NC ? c + 2 : c + 2 - NC, t2 = c + 2 < NC ? t : t + 1;
        if (t2 < d.T) {
          if (!NOHO && t2 >= 1 && !failed && !psync_reached(__builtin_amdgcn_readfirstlane(pvr[P % PL]), target(c2, t2)))
            wait_chunk(c2, t2);
          if (t2 > 0 || (DBG & 131072) == 0)
            issue_b(t2 == t ? abase : abase_n, c2, std::integral_constant<int, (P + 2) % NSLOT>{});
        }
        // poll for chunk j+2+PL (read at the top of chunk j+PL)
        const int c3 = c + 2 + PL < NC ? c + 2 + PL : c + 2 + PL - NC, t3 = c + 2 + PL < NC ? t : t + 1;
        if (!NOHO && t3 >= 1 && t3 < d.T) pvr[P % PL] = poll(c3);
      } else if constexpr (!FIRST) {
        if (c + 2 < NC) issue(c + 2, std::integral_constant<int, (P + 2) % 3>{});
      }
      // A fragment reads through asm with COUNTED waits: as C++ loads, the compiler's waitcnt
      // pass put lgkmcnt(0) before every k-tile pair, so each wait also drained the reads of
      // the NEXT k-tile issued just before it (9 exposed LDS latencies per chunk). Here the
      // reads of k-tile kt + 1 are issued at the top of kt and kt waits with lgkmcnt(2): LDS
      // returns in order, so everything but those 2 youngest reads has landed. The wait takes
      // kt's fragments as "+v" operands, so no use of them moves above it. Per-chunk bases
      // (ring slot + lane offset): the slot offset does not fit the 16-bit ds offset field.
      const unsigned ab[2] = {lds_smem + (unsigned)(P * SLOT) + (unsigned)fa[0],
                              lds_smem + (unsigned)(P * SLOT) + (unsigned)fa[1]};

      f32x4 acc_l[2][4];  // written first by k-tile 0's MFMAs (src C = 0: no zeroing writes)
      // ALT: this body's set and the previous chunk's (read by the fused stages)
      f32x4(&acc)[2][4] = [&]() -> f32x4(&)[2][4] {
        if constexpr (ALT) return accs[P & 1]; else return acc_l;
      }();
      f32x4(&accq)[2][4] = [&]() -> f32x4(&)[2][4] {
        if constexpr (ALT) return accs[(P & 1) ^ 1]; else return accp;
      }();
      // MFMAs in inline asm with explicit register classes: weights of k-tiles < KTA as AGPR
      // operands, the rest as VGPR operands, accumulators in AGPRs. With the builtin the
      // register allocator shuffled the 288 weight registers through v_accvgpr_read/mov copies
      // before every use and single-buffered the A fragments (timeline: 2.5 us per chunk of
      // MFMA work that issues in ~1 us). A fragments of k-tile kt+1 are read during kt.
      // Software pipeline: the cell epilogue of chunk c-1 (accp, cq[0]) is computed INSIDE
      // this loop, one (row-tile, row) element per k-tile, so its VALU / transcendental work
      // issues between the MFMAs (chunk 0 computes on leftovers and discards the result).
      bf16x8 a[2][2];
      float cv[2][4], gs[2][4];
      unsigned pk[2][8], hv[2][4];
      EpiMicro ms;
      // H = 512 (KT = 18, 144 MFMAs per chunk): each MFMA and one micro-stage of the carried
      // chunk's cell math are ONE asm statement. No pin asm between them, so the hazard
      // recognizer has nothing to pad: it pads (s_nop) only where an asm reads a VGPR that
      // the asm right before it wrote, and two elements are in flight with their stages
      // alternating, so a stage's producer is always >= 2 statements back. Slot m: pair
      // m / 36 (elements 2p, 2p+1), stage (m % 36) / 2 of element 2p + (m & 1). Outputs are
      // early-clobber: no stage result can share a register with the MFMA's operands.
      EpiMicro e2[2];
      auto fused_slot = [&](auto kc, auto mc) {
        constexpr int kt = decltype(kc)::value, mm = decltype(mc)::value;
        constexpr int i = mm >> 2, j = mm & 3, m = kt * 8 + mm;
        constexpr int el = 2 * (m / 36) + (m & 1), st = (m % 36) / 2, ei_ = (el >> 2) & 1, er = el & 3;
        EpiMicro& E = e2[m & 1];
        const bf16x8& A = a[kt & 1][i];
        if constexpr (m >= 144 || (DBG & 8192) != 0) {  // KT > 18: the 144 stages are placed, the rest are
                                                        // plain MFMAs (DBG 8192: timing only, no stages)
          if constexpr (ALT && kt == 0)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc[i][j]) : "v"(A), "a"(w[kt][j]));
          else if constexpr (ALT && kt < KTA)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i][j]) : "v"(A), "a"(w[kt][j]));
          else if constexpr (ALT)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i][j]) : "v"(A), "v"(w[kt][j]));
          else if constexpr (kt < KTA)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(A), "a"(w[kt][j]));
          else
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(A), "v"(w[kt][j]));
          return;
        }
#define WF_UNP(...) __VA_ARGS__
#define WF_MF(TXT, OUTS, INS)                                                                          \
  if constexpr (ALT && kt == 0)                                                                        \
    asm volatile("v_mfma_f32_16x16x32_bf16 %[c], %[a], %[b], 0\n\t" TXT                                \
                 : [c] "=&v"(acc[i][j]), WF_UNP OUTS : [a] "v"(A), [b] "a"(w[kt][j]) WF_UNP INS);    \
  else if constexpr (ALT && kt < KTA)                                                                  \
    asm volatile("v_mfma_f32_16x16x32_bf16 %[c], %[a], %[b], %[c]\n\t" TXT                             \
                 : [c] "+v"(acc[i][j]), WF_UNP OUTS : [a] "v"(A), [b] "a"(w[kt][j]) WF_UNP INS);     \
  else if constexpr (ALT)                                                                              \
    asm volatile("v_mfma_f32_16x16x32_bf16 %[c], %[a], %[b], %[c]\n\t" TXT                             \
                 : [c] "+v"(acc[i][j]), WF_UNP OUTS : [a] "v"(A), [b] "v"(w[kt][j]) WF_UNP INS);     \
  else if constexpr (kt == 0)                                                                          \
    asm volatile("v_mfma_f32_16x16x32_bf16 %[c], %[a], %[b], 0\n\t" TXT                                \
                 : [c] "=&a"(acc[i][j]), WF_UNP OUTS : [a] "v"(A), [b] "a"(w[kt][j]) WF_UNP INS);    \
  else if constexpr (kt < KTA)                                                                         \
    asm volatile("v_mfma_f32_16x16x32_bf16 %[c], %[a], %[b], %[c]\n\t" TXT                             \
                 : [c] "+a"(acc[i][j]), WF_UNP OUTS : [a] "v"(A), [b] "a"(w[kt][j]) WF_UNP INS);     \
  else                                                                                                 \
    asm volatile("v_mfma_f32_16x16x32_bf16 %[c], %[a], %[b], %[c]\n\t" TXT                             \
                 : [c] "+a"(acc[i][j]), WF_UNP OUTS : [a] "v"(A), [b] "v"(w[kt][j]) WF_UNP INS);
        if constexpr (st == 0) {
          WF_MF("v_exp_f32 %[o], %[x]", ([o] "=&v"(E.ei)), (, [x] "v"(accq[ei_][0][er])))
        } else if constexpr (st == 1) {
          WF_MF("v_exp_f32 %[o], %[x]", ([o] "=&v"(E.ef)), (, [x] "v"(accq[ei_][1][er])))
        } else if constexpr (st == 2) {
          WF_MF("v_exp_f32 %[o], %[x]", ([o] "=&v"(E.eg)), (, [x] "v"(accq[ei_][2][er])))
        } else if constexpr (st == 3) {
          WF_MF("v_exp_f32 %[o], %[x]", ([o] "=&v"(E.eo)), (, [x] "v"(accq[ei_][3][er])))
        } else if constexpr (st == 4) {
          WF_MF("v_add_f32 %[p], 1.0, %[p]\n\tv_add_f32 %[q], 1.0, %[q]", ([p] "+v"(E.ei), [q] "+v"(E.ef)), ())
        } else if constexpr (st == 5) {
          WF_MF("v_rcp_f32 %[o], %[x]", ([o] "=&v"(E.ig)), (, [x] "v"(E.ei)))
        } else if constexpr (st == 6) {
          WF_MF("v_rcp_f32 %[o], %[x]", ([o] "=&v"(E.fg)), (, [x] "v"(E.ef)))
        } else if constexpr (st == 7) {
          WF_MF("v_add_f32 %[p], 1.0, %[p]\n\tv_add_f32 %[q], 1.0, %[q]", ([p] "+v"(E.eg), [q] "+v"(E.eo)), ())
        } else if constexpr (st == 8) {
          WF_MF("v_rcp_f32 %[o], %[x]", ([o] "=&v"(E.gg)), (, [x] "v"(E.eg)))
        } else if constexpr (st == 9) {
          WF_MF("v_rcp_f32 %[o], %[x]", ([o] "=&v"(E.og)), (, [x] "v"(E.eo)))
        } else if constexpr (st == 10) {  // g = 1 - 2 r (tanh), then i * g into cn
          WF_MF("v_fma_f32 %[g], %[g], -2.0, 1.0\n\tv_mul_f32 %[c2], %[x], %[g]", ([g] "+v"(E.gg), [c2] "=&v"(E.cn)),
                (, [x] "v"(E.ig)))
        } else if constexpr (st == 11) {  // c_t = fma(f, c_{t-1}, i g); packed (i, f)
          WF_MF("v_fma_f32 %[c2], %[f], %[cp], %[c2]\n\tv_cvt_pk_bf16_f32 %[o], %[x], %[f]",
                ([c2] "+v"(E.cn), [o] "=&v"(E.p0)), (, [f] "v"(E.fg), [cp] "v"(cq[0][ei_][er]), [x] "v"(E.ig)))
        } else if constexpr (st == 12) {  // packed (g, o); 2 log2(e) c_t
          WF_MF("v_cvt_pk_bf16_f32 %[o], %[g], %[x]\n\tv_mul_f32 %[y], 0x4038aa3b, %[c2]", ([o] "=&v"(E.p1), [y] "=&v"(E.ec)),
                (, [g] "v"(E.gg), [x] "v"(E.og), [c2] "v"(E.cn)))
        } else if constexpr (st == 13) {
          WF_MF("v_exp_f32 %[p], %[p]", ([p] "+v"(E.ec)), ())
        } else if constexpr (st == 14) {
          WF_MF("v_add_f32 %[p], 1.0, %[p]", ([p] "+v"(E.ec)), ())
        } else if constexpr (st == 15) {
          WF_MF("v_rcp_f32 %[p], %[p]", ([p] "+v"(E.ec)), ())
        } else if constexpr (st == 16) {  // h = o (1 - 2 r)
          WF_MF("v_fma_f32 %[p], %[p], -2.0, 1.0\n\tv_mul_f32 %[p], %[x], %[p]", ([p] "+v"(E.ec)), (, [x] "v"(E.og)))
        } else {  // bf16(h) in the low half
          unsigned h;
          WF_MF("v_cvt_pk_bf16_f32 %[o], %[x], 0", ([o] "=&v"(h)), (, [x] "v"(E.ec)))
          cv[ei_][er] = E.cn;
          pk[ei_][2 * er] = E.p0;
          pk[ei_][2 * er + 1] = E.p1;
          hv[ei_][er] = h;
        }
#undef WF_MF
#undef WF_UNP
      };
      // A/B (WELLFLOW_PF_DBG=4096, production-correct): the round-2 C++ fragment loads
      constexpr bool CXX_FRAG = (DBG & 4096) != 0;
      if constexpr (CXX_FRAG) {
        for (int i = 0; i < 2; ++i) a[0][i] = *reinterpret_cast<const bf16x8*>(smem + P * SLOT + i * 2048 + fa[0]);
      } else {
        asm volatile("ds_read_b128 %0, %1" : "=v"(a[0][0]) : "v"(ab[0]) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(a[0][1]) : "v"(ab[0]) : "memory");
      }
      if constexpr ((DBG & 32) != 0) {
        a[1][0] = a[0][0];
        a[1][1] = a[0][1];
      }
      static_for<0, KT>([&](auto kc) {
        constexpr int kt = decltype(kc)::value;
        if constexpr ((DBG & 16) != 0 && kt < 20) {  // timeline: k-tile starts of chunk 3, slots 42..
          if (c == 3) stamp(t, 42 + kt);
        }
        if constexpr (CXX_FRAG) {
          if constexpr (kt + 1 < KT)
            for (int i = 0; i < 2; ++i)
              a[(kt + 1) & 1][i] = *reinterpret_cast<const bf16x8*>(smem + P * SLOT + ((kt + 1) >> 1) * 4096 +
                                                                     i * 2048 + fa[(kt + 1) & 1]);
        } else if constexpr (kt + 1 < KT && !(DBG & 32)) {  // DBG & 32: timing only, no fragment reads
          constexpr int o = ((kt + 1) >> 1) * 4096;
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[(kt + 1) & 1][0]) : "v"(ab[(kt + 1) & 1]), "i"(o)
                       : "memory");
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[(kt + 1) & 1][1]) : "v"(ab[(kt + 1) & 1]),
                       "i"(o + 2048) : "memory");
          asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(a[kt & 1][0]), "+v"(a[kt & 1][1]) :: "memory");
        } else if constexpr (!CXX_FRAG) {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[kt & 1][0]), "+v"(a[kt & 1][1]) :: "memory");
        }
        static_for<0, 8>([&](auto mc) {
          constexpr int i = decltype(mc)::value >> 2, j = decltype(mc)::value & 3;
          if constexpr (FIRST) {  // no carried chunk: plain MFMAs, next chunks' pieces in between
            if constexpr (kt == 0)
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
                           : "=&a"(acc[i][j]) : "v"(a[kt & 1][i]), "a"(w[kt][j]));
            else if constexpr (kt < KTA)
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(a[kt & 1][i]), "a"(w[kt][j]));
            else
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(a[kt & 1][i]), "v"(w[kt][j]));
            if constexpr (decltype(mc)::value == 0)  // piece kt of chunks 1, 2 (KS pieces each)
              issue_piece(1 + kt / KS, std::integral_constant<int, 1 + kt / KS>{}, kt % KS);
            return;
          }
          if constexpr (FUSED) {
            fused_slot(kc, mc);
            return;
          }
          if constexpr (!(DBG & 2)) {
            if constexpr (kt == 0)  // accumulator := A B (inline-constant 0 as src C)
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
                           : "=&a"(acc[i][j]) : "v"(a[kt & 1][i]), "a"(w[kt][j]));
            else if constexpr (kt < KTA)
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(a[kt & 1][i]), "a"(w[kt][j]));
            else
              asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(a[kt & 1][i]), "v"(w[kt][j]));
          }
          if constexpr (!(DBG & 128)) {
            // micro-stages of the carried chunk's cell math, one issue-slot's worth (<= 8
            // cycles: one transcendental or two plain VALU) in each MFMA's shadow:
            // stage q of 144 (8 elements x 18) goes after MFMA slot q * 8KT / 144
            constexpr int S = 8 * KT, m = kt * 8 + decltype(mc)::value;
            constexpr int qlo = (m * 144 + S - 1) / S, qhi = ((m + 1) * 144 + S - 1) / S;
            static_for<qlo, qhi>([&](auto qc) {
              constexpr int q = decltype(qc)::value;
              epi_micro(std::integral_constant<int, q % 18>{}, q / 18 >> 2, (q / 18) & 3, ms, cv, pk, hv);
            });
          }
        });
        if constexpr ((DBG & 128) != 0) {
          // 16 half-elements spread evenly over the KT k-tiles (half q at k-tile q * KT / 16)
          static_for<0, 16>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            if constexpr (q * KT / 16 == kt) epi_half(q & 1, q >> 3, (q >> 1) & 3, cv, gs, pk, hv);
          });
        }
        if constexpr (KT >= 16 && (DBG & 64)) {  // chunk c-1's stores and publish in this loop's shadow
          if constexpr (kt == 8) {
            if (c > 0) epi_h(hv);
          }
          if constexpr (kt >= 9 && kt <= 14) {
            if (c > 0) epi_cs(c - 1, kt - 9, cv, pk);
          }
          if constexpr (kt == 16) {
            if (c > 0) publish(c - 1);
          }
        }
        // The MFMAs are inline asm, so the compiler knows neither their latency nor that they
        // still read this k-tile's A fragments after issue: keep those registers allocated to
        // the end of the k-tile, so no micro-stage result lands in them under an MFMA in
        // flight (it did: a v_accvgpr_read into SrcA one instruction after the MFMA, wrong h
        // at H = 128 / 256).
        asm volatile("" ::"v"(a[kt & 1][0]), "v"(a[kt & 1][1]));
      });
      // the epilogue reads the accumulators with VALU: cover the last MFMAs' pipeline
      // (the compiler pads nothing after inline asm). The accumulators are operands of the
      // padding, so no read of them (the accp copy, or the drain's cell math at NC = 1) can
      // be scheduled above it: the compiler sees an inline-asm MFMA's result as ready at
      // once and had put v_accvgpr_reads 2 instructions behind the last MFMAs (tools/mfma_war.py).
      if constexpr (ALT)  // the set's next reader is the next body's first stage: one pad is plenty
        asm volatile("s_nop 7"
                     : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[0][2]), "+v"(acc[0][3]), "+v"(acc[1][0]),
                       "+v"(acc[1][1]), "+v"(acc[1][2]), "+v"(acc[1][3])
                     :
                     : "memory");
      else
        asm volatile("s_nop 7\n\ts_nop 7"
                     : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[0][2]), "+a"(acc[0][3]), "+a"(acc[1][0]),
                       "+a"(acc[1][1]), "+a"(acc[1][2]), "+a"(acc[1][3])
                     :
                     : "memory");
      if constexpr ((DBG & 16) != 0) {  // MFMA completion: consume a result before stamping
        float sink = acc[1][3][3];
        asm volatile("" ::"v"(sink));
        stamp(t, 4 + 5 * c);
      }
      if constexpr (SPLIT) {
        if (t > 0 || c > 0) {
          const bool prv = c == 0;  // the previous step's last chunk
          epi_store_split(prv ? NC - 1 : c - 1, prv ? cnext_p : cnext, prv ? St_p : St, prv ? xh_rsrc_p : xh_rsrc,
                          cv, pk, hv);
          stamp(t, 5 + 5 * c);
        }
      } else if constexpr (KT >= 16 && (DBG & 64)) {
        if (c > 0) rotate(cv);
      } else if (c > 0 && (DBG & 16384) == 0) {  // DBG 16384: timing only, no stores / publish
        epi_store(c - 1, cv, pk, hv);
        stamp(t, 5 + 5 * c);
        publish(c - 1);
      }
      if constexpr (!ALT) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) accp[i][j] = acc[i][j];
      }
      stamp(t, 6 + 5 * c);
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    using S2 = std::integral_constant<int, 2>;
    using S3 = std::integral_constant<int, 3>;
    using NF = std::false_type;
    if constexpr (SPLIT) {
      if (t == 0) {  // chunks 0 and 1 of step 0 (XH[0] = [x_0 | 1 | h_-1 = 0] is written before the launch)
        issue_b0(abase, 0, S0{});
        issue_b0(abase, 1, S1{});
      }
      for (int c = 0; c < NC; c += 4) {
        chunk(c, S0{}, NF{});
        chunk(c + 1, S1{}, NF{});
        chunk(c + 2, S2{}, NF{});
        chunk(c + 3, S3{}, NF{});
      }
      if (t == d.T - 1) {  // drain: the last chunk's epilogue (h_T is the regression head's input)
        float cv[2][4];
        unsigned pk[2][8], hv[2][4];
#pragma unroll
        for (int e = 0; e < 8; ++e) epi_elem(e >> 2, e & 3, cv, pk, hv);
        epi_store_split(NC - 1, cnext, St, xh_rsrc, cv, pk, hv);
      }
    } else {
      if constexpr (PF01) {
        chunk(0, S0{}, std::true_type{});
        for (int c = 1; c < NC; c += 3) {
          chunk(c, S1{}, NF{});
          if (c + 1 < NC) chunk(c + 1, S2{}, NF{});
          if (c + 2 < NC) chunk(c + 2, S0{}, NF{});
        }
      } else {
        for (int c = 0; c < NC; c += 3) {
          chunk(c, S0{}, NF{});
          if (c + 1 < NC) chunk(c + 1, S1{}, NF{});
          if (c + 2 < NC) chunk(c + 2, S2{}, NF{});
        }
      }
      {  // drain: the last chunk's epilogue
        float cv[2][4];
        unsigned pk[2][8], hv[2][4];
#pragma unroll
        for (int e = 0; e < 8; ++e) epi_elem(e >> 2, e & 3, cv, pk, hv);
        // h first (the only bytes other workgroups read in this launch), then the C / S stores,
        // so the step-top hand-off drains only the h store (vmcnt(NSTORE - 1)) and the last
        // chunk's C / S stores complete behind the hand-off instead of in front of it
        // Deferring these six stores past the next step's hand-off (after chunk 0's loop, which
        // stores nothing) measured neutral to worse: 1470-1486 us deferred vs 1454-1482 here
        // (profiles/r3/ab_defer_drain_stores.txt). The write burst is not on the critical path.
        if constexpr ((DBG & 65536) != 0) {  // A/B: the round-2 order (stores, then h)
          epi_store(NC - 1, cv, pk, hv);
          publish(NC - 1);
        } else {
          epi_h(hv);
          publish(NC - 1);
          if constexpr (!(DBG & 4)) {
#pragma unroll
            for (int k = 0; k < 6; ++k) epi_cs(NC - 1, k, cv, pk);
          }
          rotate(cv);
        }
      }
    }
    cnext_p = cnext;
    St_p = St;
    xh_rsrc_p = xh_rsrc;
  }
  // completion count: a workgroup none of whose waves failed a hand-off adds T to DONE; a
  // failure leaves DONE short of EXPECT, which the host check reports
  wait_vmcnt<0>();
  asm volatile("ds_write_b32 %0, %1" ::"v"(flag_lds + 16 + 4 * wid), "v"(failed) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (threadIdx.x == 0) {
    u32x4 fw;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(fw) : "v"(flag_lds + 16) : "memory");
    if ((fw[0] | fw[1] | fw[2] | fw[3]) == 0u) pguard_done(stat, (unsigned)d.T);
  }
}

template <int KT, int NC>
static int launch_pf(bf16_t* XH, const bf16_t* Wp, bf16_t* Cst, bf16_t* S, unsigned* sync, unsigned* stat, int grid,
                     LstmDims d, hipStream_t s) {
  const void* f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC>);
#ifdef WF_DIAG  // A/B and timing-only variants: diagnostic builds only (WELLFLOW_DIAG_BUILD=1)
  const void* const prod = f;
  if constexpr (KT == 18 && NC == 8) {
    if constexpr (WF_DV(4096)) { if (d.dbg == 4096) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 4096>); }  // C++ fragments
    if constexpr (WF_DV(65536)) { if (d.dbg == 65536) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 65536>); }  // round-2 store order
    if constexpr (WF_DV(2)) { if (d.dbg == 2) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 2>); }
    if constexpr (WF_DV(4)) { if (d.dbg == 4) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 4>); }
    if constexpr (WF_DV(14)) { if (d.dbg == 14) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 14>); }
    if constexpr (WF_DV(16)) { if (d.dbg == 16) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 16>); }
    if constexpr (WF_DV(48)) { if (d.dbg == 48) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 48>); }
    if constexpr (WF_DV(64)) { if (d.dbg == 64) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 64>); }  // stores inside the loop
    if constexpr (WF_DV(1024)) { if (d.dbg == 1024) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 1024>); }  // chunk 1 at the step top
    if constexpr (WF_DV(512)) { if (d.dbg == 512) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 512>); }  // pinned micro-stages
    if constexpr (WF_DV(128)) { if (d.dbg == 128) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 128>); }  // half-element epilogue
    if constexpr (WF_DV(8192)) { if (d.dbg == 8192) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 8192>); }  // no cell math in the loop
    if constexpr (WF_DV(16384)) { if (d.dbg == 16384) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 16384>); }  // no stores / publish
    if constexpr (WF_DV(24576)) { if (d.dbg == 24576) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 24576>); }  // neither
    if constexpr (WF_DV(256)) { if (d.dbg == 256) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 256>); }  // per-wave h pieces
    if constexpr (WF_DV(2048)) { if (d.dbg == 2048) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 2048>); }  // AGPR accumulators
    if constexpr (WF_DV(262144)) { if (d.dbg == 262144) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 262144>); }  // round-5 publish delay
    if constexpr (WF_DV(264192)) { if (d.dbg == 264192) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 264192>); }  // the round-5 kernel
    if constexpr (WF_DV(8)) { if (d.dbg == 8) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 8>); }  // poll two chunks ahead
    if constexpr (WF_DV(524288)) { if (d.dbg == 524288) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 524288>); }  // no hand-off
    if constexpr (WF_DV(663584)) { if (d.dbg == 663584) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 663584>); }  // bare MFMAs + stores, no hand-off
    if constexpr (WF_DV(663588)) { if (d.dbg == 663588) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 663588>); }  // bare MFMAs, h staging only
    if constexpr (WF_DV(32)) { if (d.dbg == 32) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 32>); }  // no fragment reads
    if constexpr (WF_DV(8224)) { if (d.dbg == 8224) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 8224>); }  // neither cell math nor fragment reads
    if constexpr (WF_DV(131072)) { if (d.dbg == 131072) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 131072>); }  // no LDS-DMA
    if constexpr (WF_DV(139296)) { if (d.dbg == 139296) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 139296>); }  // bare MFMAs + hand-off + stores
    if constexpr (WF_DV(139300)) { if (d.dbg == 139300) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 139300>); }  // bare MFMAs + hand-off, no C/S stores
    if constexpr (WF_DV(32768)) { if (d.dbg == 32768) f = reinterpret_cast<const void*>(&lstm_fwd_persistent_kernel<KT, NC, 32768>); }  // round-2 S slots
  }
  // a requested variant that this build did not compile must not time the production kernel
  // under its name (bits 0 and 20-22 are runtime switches, not variants)
  if ((d.dbg & 0xFFFFE) != 0 && f == prod) return -(int)hipErrorInvalidDeviceFunction;
#endif
  void* args[] = {&XH, &Wp, &Cst, &S, &sync, &stat, &d};
  return persistent_launch(f, grid, args, s);  // persistent_launch.h: residency check + plain launch
}

}  // namespace wf
