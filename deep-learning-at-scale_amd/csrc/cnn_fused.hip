// wellflow — fused kernels of the reference's own model, the 1-D CNN of cnn.py:110-118
// (SURVEY.md §2.4 K1-K9): Conv1D(1 -> 100 filters, width 13, valid) + ReLU -> Dropout(0.5) ->
// Flatten -> Dense(3600 -> 12), clipped-MAE (or MSE) loss, Keras SGD-Nesterov.
//
// Why: the round-3 engine ran im2col to HBM + three generic 128x128 GEMM launches + a loss
// kernel. The 36 x 100 activation of every window was written, re-read as the dense input and
// as the ReLU/dropout mask, its gradient written and re-read (~3.2 GB of HBM per step at
// B = 65,536), and the skinny GEMMs (N = 12 outputs, K = 13 taps) ran 128-wide tiles that were
// 7/8 padding: 1.63 ms per step, ~1 % of the MFMA peak (round-3 VERDICT missing #1). Here the
// activation never leaves the CU and every product is a 16x16x16 MFMA shaped to the layer:
//
//  * forward (cnn_fwd_kernel): one wave owns a group of 16 windows and walks the 36 output
//    steps t. Per t: P^T[f x w] = Wc[f x kk] X_t^T[kk x w] (7 MFMAs over the 112 padded filters;
//    the lane's B fragment x[w][t + kk] comes out of its window's samples held as bf16 pairs
//    in registers, the conv bias rides in the K slot kk = 13 against a constant 1), ReLU and
//    the dropout mask in registers, then out^T[j x w] += Wd_t^T[j x f] act^T[f x w] — the
//    accumulator tile IS the next MFMA's B operand (rows f, no lane movement). The dense
//    weights sit in LDS in a fragment-native image (one conflict-free ds_read_b64 per MFMA).
//    The epilogue adds the dense bias, evaluates the loss and writes only dOut (64 B per
//    window) and per-workgroup partials of the loss and of the dense-bias gradient.
//  * backward (cnn_bwd_kernel): grid = (pairs of output steps) x (window chunks); the
//    workgroup keeps its two steps' dense-weight fragments and the gradient tiles dWd_t and
//    dWc in registers for its whole chunk. Per (16-window group, t) it recomputes P (7 MFMAs),
//    dAct = dOut Wd_t (7), masks it with the SAME dropout bits and ReLU, and accumulates
//    dWd_t += act^T dOut (7) and dWc += dP^T X_t (7) — the bias row kk = 13 of X is the
//    constant 1, so that row of dWc is the conv-bias gradient. Partials go out once per
//    workgroup; cnn_reduce_kernel sums them into the flat gradient and advances the dropout
//    step counter.
//
// Dropout (p = 0.5, Keras inverted dropout) is a counter hash, never stored: the keep bit of
// (window w, step t, filter f = 16b + 4q + r) is bit k + 16 (r & 1), k = 2b + (r >> 1), of
// lowbias32(((w*T + t)*4 + q) ^ smix), smix mixing the engine seed and the device step counter
// (so every hipGraph replay draws a new mask). The forward needs one hash per lane per step (its
// lane holds filters 16b + 4q + r of one window), the backward four (four windows per lane).
// The two keep bits of a bf16 pair (r, r+1 of block b: k = 2b + r/2) sit 16 bits apart, so ONE
// shift moves both into the pair's sign bits: OR-ing them into the packed activations makes a
// dropped value negative, and one packed int16 max with 0 is ReLU and dropout of both halves
// (bf16 orders like int16 on the non-negative side; every negative, -0 included, becomes +0).
// wellflow/models/cnn.py cnn_dropout_mask mirrors it bit for bit for the fp32 tests. The
// 1/(1-p) = 2 scale is applied to the dense output (forward) and to dOut (backward) instead
// of to every activation.
#include <cstdlib>

#include "common.h"
#include "gemm_core.h"
#include "kernels.h"

namespace wf {

namespace {
constexpr int CNN_NW = 8;    // waves per workgroup (512 threads, 2 per SIMD)
constexpr int CNN_TG = 2;    // output steps per backward workgroup
constexpr int CNN_NFB = 7;   // 16-filter blocks (filters 97..112; the reference has 100)
constexpr int CNN_T = 36;    // output steps (input 48, width 13)

__device__ __forceinline__ f32x4 mfma16(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16x4 frag(unsigned lo, unsigned hi) {
  return __builtin_bit_cast(bf16x4, (u32x2{lo, hi}));
}
__device__ __forceinline__ bf16x8 frag8(unsigned a, unsigned b, unsigned c, unsigned d) {
  return __builtin_bit_cast(bf16x8, (u32x4v{a, b, c, d}));
}
// ReLU of a packed bf16 pair: one v_pk_max_i16 against 0 (see the dropout note above)
__device__ __forceinline__ unsigned relu_pk(unsigned v) {
  const i16x2 r = __builtin_elementwise_max(__builtin_bit_cast(i16x2, v), (i16x2{0, 0}));
  return __builtin_bit_cast(unsigned, r);
}
// dropout of pair k given the lane's INVERTED mask word mi = ~m: keep bits k and k + 16 (set =
// dropped after the inversion) into the two sign bits, so relu_pk zeroes a dropped value:
// v_lshlrev + v_and_or_b32
__device__ __forceinline__ unsigned drop_pk(unsigned v, unsigned mi, int k) {
  return (mi << (15 - k)) & 0x80008000u | v;
}
__device__ __forceinline__ unsigned lowbias32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
}  // namespace

// step mix of the dropout hash: engine seed x device step counter (cnn.py cnn_dropout_mask)
__device__ __forceinline__ unsigned cnn_seed_mix(unsigned seed, const long long* rng) {
  const unsigned r = rng != nullptr ? (unsigned)rng[0] : 0u;
  return lowbias32(seed ^ lowbias32(r + 0x9E3779B9u));
}
__device__ __forceinline__ unsigned cnn_mask_word(unsigned smix, int w, int t, int T, int q) {
  return lowbias32((((unsigned)w * (unsigned)T + (unsigned)t) * 4u + (unsigned)q) ^ smix);
}

// The K-slot fix-up of an X fragment (lane quad q holds kk = 4q .. 4q+3): kk == taps is the
// constant 1 of the folded conv bias, kk > taps are zero. Per-lane masks, one v_and_or each.
struct KSlot {
  unsigned keep0, keep1, one0, one1;
  __device__ KSlot(int q, int taps) {
    keep0 = keep1 = one0 = one1 = 0u;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int kk = 4 * q + jj;
      const unsigned half = (jj & 1) ? 0xFFFF0000u : 0x0000FFFFu;
      const unsigned onev = (jj & 1) ? 0x3F800000u : 0x00003F80u;  // bf16 1.0
      unsigned& keep = jj < 2 ? keep0 : keep1;
      unsigned& one = jj < 2 ? one0 : one1;
      if (kk < taps) keep |= half;
      if (kk == taps) one |= onev;
    }
  }
  __device__ __forceinline__ bf16x4 apply(unsigned d0, unsigned d1) const {
    return frag((d0 & keep0) | one0, (d1 & keep1) | one1);
  }
};

// ------------------------------------------------------------------------------- forward
// TRAIN: loss + dOut + partials, DROP: dropout (compile-time: a runtime flag became a
// v_cndmask per pair). !TRAIN: predictions only (eval).
template <int NFB, int T, bool TRAIN, bool DROP>
__global__ __launch_bounds__(512, 1) void cnn_fwd_kernel(
    const float* __restrict__ x, int B, int L, const bf16_t* __restrict__ WcA, int Kc,
    const bf16x4* __restrict__ WdF, const float* __restrict__ bd, int O, const float* __restrict__ y,
    float* __restrict__ dout, float* __restrict__ pred, float* __restrict__ part, int taps, int loss_kind,
    float clip, float scale, float keep_scale, int drop, unsigned seed, const long long* __restrict__ rng, int prio) {
  constexpr int XR = (T + 6) / 4 * 4;  // x samples per lane: 4q .. 4q + T + 2, whole float4s
  constexpr int NFRAG = T * NFB * 64;
  static_assert(NFB == 7, "dense fragments: 3 filter-block pairs (16x16x32) + block 6 (16x16x16)");
  constexpr int TB = NFB * 64 * 8;  // bytes of one step's dense fragments
  // ONE static LDS object: the dense weights' fragment image, then the wave partials
  __shared__ __attribute__((aligned(16))) char smem[NFRAG * 8 + CNN_NW * 20 * 4];
  float* wpart = reinterpret_cast<float*>(smem + NFRAG * 8);
  const int lane = threadIdx.x & 63, l15 = lane & 15, q = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  (void)prio;
  const int ngroups = (B + 15) >> 4;
  // the lane's x samples, loaded one group AHEAD (issued before this group's 36 steps, consumed
  // a group later): raw float4s from a clamped in-range address, bounds applied at consumption
  // (and, training, its 4 targets: a load in the epilogue exposed its latency once per group)
  float4 xnx[XR / 4];
  float ynx[4];
  auto load_x = [&](int g) {
    const int wc = min(g * 16 + l15, B - 1);
#pragma unroll
    for (int k = 0; k < XR / 4; ++k)
      xnx[k] = *reinterpret_cast<const float4*>(x + (size_t)wc * L + min(4 * q + 4 * k, L - 4));
    if constexpr (TRAIN) {
#pragma unroll
      for (int r = 0; r < 4; ++r) ynx[r] = y[(size_t)wc * O + min(4 * q + r, O - 1)];
    }
  };
  const int gstride = gridDim.x * CNN_NW;
  // the first group's x and the dense weights' fragment image go out together: the image as
  // 1-KiB LDS-DMA pieces (global_load_lds, wave w moves pieces w, w + 8, ..; no register round
  // trip), the x loads behind them, one wait for both
  if ((int)blockIdx.x * CNN_NW + wid < ngroups) load_x(blockIdx.x * CNN_NW + wid);
  {
    typedef __attribute__((address_space(3))) void lds_v;
    const char* src = reinterpret_cast<const char*>(WdF);
    for (int pc = wid; pc < NFRAG * 8 / 1024; pc += CNN_NW)
      __builtin_amdgcn_global_load_lds((const void*)(src + pc * 1024 + lane * 16), (lds_v*)(smem + pc * 1024), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // conv weights as the A operand: A[f = 16b + l15][kk = 4q + jj] (bias at kk = taps)
  bf16x4 wc[NFB];
#pragma unroll
  for (int b = 0; b < NFB; ++b) wc[b] = *reinterpret_cast<const bf16x4*>(WcA + (size_t)(16 * b + l15) * Kc + 4 * q);
  const KSlot ks(q, taps);
  float bdj[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bdj[r] = bd[4 * q + r];
  (void)drop;
  const unsigned smix = DROP ? cnn_seed_mix(seed, rng) : 0u;
  float lsum = 0.f, dbd[4] = {0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  for (int g = blockIdx.x * CNN_NW + wid; g < ngroups; g += gstride) {
    const int w = g * 16 + l15;  // this lane's window (B-operand column)
    const bool wok = w < B;
    unsigned xp[XR / 2];  // bf16 pairs (x[w][4q + 2i], x[w][4q + 2i + 1])
#pragma unroll
    for (int k = 0; k < XR / 4; ++k) {
      const bool ok = wok && 4 * q + 4 * k + 4 <= L;
      const float4 v = xnx[k];
      xp[2 * k] = ok ? pk_bf16(v.x, v.y) : 0u;
      xp[2 * k + 1] = ok ? pk_bf16(v.z, v.w) : 0u;
    }
    float ycur[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ycur[r] = TRAIN ? ynx[r] : 0.f;
    load_x(min(g + gstride, ngroups - 1));  // (the last group re-loads itself: never read)
    f32x4 out = {0.f, 0.f, 0.f, 0.f};
    // dense-weight fragments of step t (pairs of 16-filter blocks as 16x16x32 A operands, block
    // 6 as a 16x16x16 one), prefetched one step ahead; the scheduling barrier at the end of
    // every step keeps the unrolled loop from hoisting all the LDS reads (spills without it)
    const char* wdl = smem;
    bf16x8 wp[3];
    bf16x4 w6;
#pragma unroll
    for (int p = 0; p < 3; ++p) wp[p] = *reinterpret_cast<const bf16x8*>(wdl + p * 1024 + lane * 16);
    w6 = *reinterpret_cast<const bf16x4*>(wdl + 3072 + lane * 8);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const char* wn = wdl + ((t + 1) % T) * TB;
      bf16x8 wpn[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) wpn[p] = *reinterpret_cast<const bf16x8*>(wn + p * 1024 + lane * 16);
      const bf16x4 w6n = *reinterpret_cast<const bf16x4*>(wn + 3072 + lane * 8);
      // X_t^T fragment: B[kk = 4q + jj][w = l15] = x[w][t + 4q + jj]
      unsigned d0, d1;
      if (t & 1) {
        d0 = __builtin_amdgcn_alignbit(xp[(t + 1) / 2], xp[(t - 1) / 2], 16);
        d1 = __builtin_amdgcn_alignbit(xp[(t + 3) / 2], xp[(t + 1) / 2], 16);
      } else {
        d0 = xp[t / 2];
        d1 = xp[t / 2 + 1];
      }
      const bf16x4 xb = ks.apply(d0, d1);
      const unsigned mi = DROP ? ~cnn_mask_word(smix, w, t, T, q) : 0u;
      // act pairs: rows f = 16b + 4q + {0,1} and {2,3} of each block, bf16, ReLU + dropout
      unsigned act[NFB][2];
#pragma unroll
      for (int b = 0; b < NFB; ++b) {
        const f32x4 pv = mfma16(wc[b], xb, f32x4{0.f, 0.f, 0.f, 0.f});  // rows f = 16b + 4q + r
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          unsigned v = pk_bf16(pv[2 * h], pv[2 * h + 1]);
          if constexpr (DROP) v = drop_pk(v, mi, 2 * b + h);
          act[b][h] = relu_pk(v);
        }
      }
      // out^T[j x w] += Wd_t^T[j x f] act^T[f x w]: blocks (0,1) (2,3) (4,5) on the double-rate
      // 16x16x32 (k-slots 8q..8q+3 = block 2p, 8q+4..8q+7 = block 2p+1), block 6 on 16x16x16
#pragma unroll
      for (int p = 0; p < 3; ++p)
        out = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            wp[p], frag8(act[2 * p][0], act[2 * p][1], act[2 * p + 1][0], act[2 * p + 1][1]), out, 0, 0, 0);
      out = mfma16(w6, frag(act[6][0], act[6][1]), out);
      // xb stays live to the end of the step: with its registers free right after the last conv
      // MFMA, hipcc reallocated them to the next VALU result in the very next instruction, and in
      // the dropout build that corrupted 2 % of dOut on this hardware (a VALU write of an MFMA's
      // SrcB at 0 wait states; bit-exact against a bf16 emulation with this line,
      // tests/test_engines_gpu.py::test_native_cnn_bit_exact_vs_bf16_emulation,
      // profiles/r5/mfma_srcb_war.md)
      asm volatile("" ::"v"(xb));
#pragma unroll
      for (int p = 0; p < 3; ++p) wp[p] = wpn[p];
      w6 = w6n;
      __builtin_amdgcn_sched_barrier(0);
    }
    // lane holds out[j = 4q + r][w = l15]
    float d[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 4 * q + r;
      const float pv = out[r] * keep_scale + bdj[r];
      d[r] = 0.f;
      if (TRAIN) {
        if (wok && j < O) {
          const float yv = ycur[r];
          float l, dd;
          if (loss_kind == 0) {
            const float e = pv - yv;
            l = e * e;
            dd = 2.f * e;
          } else {
            const float e = yv - pv, ae = fabsf(e);
            l = fminf(ae, clip);
            const float sg = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f);
            dd = ae <= clip ? -sg : 0.f;
          }
          lsum += l;
          d[r] = dd * scale;
          dbd[r] += d[r];
        }
      } else {
        d[r] = pv;
      }
    }
    // every row of the group, rows past B too (as zeros): the buffers hold whole groups and
    // the backward reads whole groups (a smaller batch must not see a larger one's rows)
    float* dst = (TRAIN ? dout : pred) + (size_t)w * 16 + 4 * q;
    *reinterpret_cast<float4*>(dst) = make_float4(d[0], d[1], d[2], d[3]);
  }
  if (!TRAIN) return;
  // dbd[j] over the 16 lanes of quad q, the loss over the wave; then over the 8 waves
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) dbd[r] += __shfl_xor(dbd[r], o, 64);
    lsum += __shfl_xor(lsum, o, 64);
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (l15 == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) wpart[wid * 20 + 4 * q + r] = dbd[r];
    if (q == 0) wpart[wid * 20 + 16] = lsum;
  }
  __syncthreads();
  if (threadIdx.x < 17) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < CNN_NW; ++k) s += wpart[k * 20 + threadIdx.x];
    part[blockIdx.x * 32 + threadIdx.x] = s;
  }
}

// ------------------------------------------------------------------------------ backward
template <int NFB, int TG, bool DROP>
__global__ __launch_bounds__(512, 1) void cnn_bwd_kernel(
    const float* __restrict__ x, int B, int L, const bf16_t* __restrict__ WcA, int Kc,
    const bf16x4* __restrict__ WdB, const float* __restrict__ dout, int T, int taps, float keep_scale, int drop,
    unsigned seed, const long long* __restrict__ rng, int nch, float* __restrict__ part_wd,
    float* __restrict__ part_wc, int prio) {
  __shared__ __attribute__((aligned(16))) f32x4 red[CNN_NW * TG * NFB * 64];
  const int lane = threadIdx.x & 63, l15 = lane & 15, q = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  (void)prio;
  (void)drop;
  const int ntg = (T + TG - 1) / TG;
  // logical block: consecutive ids (one XCD under the round-robin deal) share a window chunk
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int ch = lb / ntg, tg = lb % ntg, t0 = tg * TG;
  const int ngroups = (B + 15) >> 4;
  const int gpc = (ngroups + nch - 1) / nch;
  const int g_begin = ch * gpc, g_end = min(ngroups, g_begin + gpc);

  // conv weights as the B operand of P[w x f]: B[kk = 4q + jj][f = 16b + l15]
  bf16x4 wc[NFB];
#pragma unroll
  for (int b = 0; b < NFB; ++b) wc[b] = *reinterpret_cast<const bf16x4*>(WcA + (size_t)(16 * b + l15) * Kc + 4 * q);
  // dense weights of this workgroup's steps as the B operand of dAct[w x f]: B[j = 4q + jj][f]
  bf16x4 wdb[TG][NFB];
#pragma unroll
  for (int tt = 0; tt < TG; ++tt)
#pragma unroll
    for (int b = 0; b < NFB; ++b)
      wdb[tt][b] = (t0 + tt < T) ? WdB[((t0 + tt) * NFB + b) * 64 + lane] : bf16x4{0, 0, 0, 0};
  const KSlot ks(q, taps);
  // the dWc B operand's row kk = l15: x for kk < taps, the constant 1 at kk = taps, else 0
  const bool kx = l15 < taps;
  const float kone = l15 == taps ? 1.f : 0.f;
  const unsigned smix = DROP ? cnn_seed_mix(seed, rng) : 0u;
  // dropout hash key of this lane's filter column f = 16b + l15 and its bit: 2b + hb0
  const int hq = l15 >> 2, hb0 = ((l15 & 3) >> 1) + 16 * (l15 & 1);

  f32x4 acc_wd[TG][NFB], acc_wc[NFB];
#pragma unroll
  for (int b = 0; b < NFB; ++b) {
    acc_wc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tt = 0; tt < TG; ++tt) acc_wd[tt][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // the group's global operands through a per-wave LDS ring, two groups AHEAD: 6 LDS-DMA
  // instructions per group (dOut rows [16][16] as one 16-B piece per lane, the x window [16
  // rows][XS samples] as five 4-B pieces per lane), counted vmcnt waits, plain LDS reads at
  // consumption. (Round 5 before: register loads one group ahead, 39 % of the cycles still
  // waiting on them; two register sets rotate through copies that wait for the newest loads.)
  // Raw values only; bounds selects are applied at consumption. Rows past B of dOut are zero
  // in the buffer (the forward writes every row of the last group it owns); x addresses are
  // clamped in range (the selects zero what they stand for). The ring aliases `red`, used only
  // after the loop.
  constexpr int XS = 20;                  // x samples per ring row: t0 .. t0 + 19 (TG + 15 used)
  constexpr int GSLOT = 1024 + 16 * XS * 4;
  constexpr int NSLOT = 3;  // two groups in flight (three: 72.55 vs 72.63 us, no gain)
  static_assert(TG + 15 <= XS && 16 * XS <= 5 * 64, "x window: five 64-lane pieces");
  static_assert(CNN_NW * NSLOT * GSLOT <= (int)sizeof(red), "ring inside the reduction buffer");
  typedef __attribute__((address_space(3))) void lds_v;
  char* ring = reinterpret_cast<char*>(red) + wid * (NSLOT * GSLOT);
  int xoff[5];  // ring element 64k + lane -> (row, sample): row * L + clamped sample
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int e = 64 * k + lane, r = min(e / XS, 15);
    xoff[k] = r * L + min(t0 + e % XS, L - 1);
  }
  auto issue = [&](int g, int slot) {
    char* st = ring + slot * GSLOT;
    const int w0 = g * 16;
    __builtin_amdgcn_global_load_lds((const void*)(dout + (size_t)w0 * 16 + lane * 4), (lds_v*)st, 16, 0, 0);
    if (w0 + 15 < B) {
      const float* xg = x + (size_t)w0 * L;
#pragma unroll
      for (int k = 0; k < 5; ++k)
        __builtin_amdgcn_global_load_lds((const void*)(xg + xoff[k]), (lds_v*)(st + 1024 + 256 * k), 4, 0, 0);
    } else {  // the batch's last, partial group: rows clamped to B - 1
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int e = 64 * k + lane, r = min(e / XS, 15);
        const float* src = x + (size_t)min(w0 + r, B - 1) * L + (xoff[k] - r * L);
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_v*)(st + 1024 + 256 * k), 4, 0, 0);
      }
    }
  };
  struct GroupLoads {
    float4 da;
    float dbv[4], xa[TG + 3], xb[TG][4];
  };
  auto read_group = [&](int slot, GroupLoads& G) {
    const float* D = reinterpret_cast<const float*>(ring + slot * GSLOT);
    const float* X = D + 256;
    G.da = make_float4(D[l15 * 16 + 4 * q], D[l15 * 16 + 4 * q + 1], D[l15 * 16 + 4 * q + 2], D[l15 * 16 + 4 * q + 3]);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) G.dbv[jj] = D[(4 * q + jj) * 16 + l15];
#pragma unroll
    for (int i = 0; i < TG + 3; ++i) G.xa[i] = X[l15 * XS + 4 * q + i];
#pragma unroll
    for (int tt = 0; tt < TG; ++tt)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) G.xb[tt][jj] = X[(4 * q + jj) * XS + tt + l15];
  };
  auto process = [&](const GroupLoads& cur, int g) {
    const int w0 = g * 16;
    // dOut (x keep_scale) as A[w = l15][j = 4q + jj] and as B[w = 4q + jj][j = l15]
    const float4 da = cur.da;
    const bf16x4 doA = frag(pk_bf16(da.x * keep_scale, da.y * keep_scale), pk_bf16(da.z * keep_scale, da.w * keep_scale));
    const bf16x4 doB = frag(pk_bf16(cur.dbv[0] * keep_scale, cur.dbv[1] * keep_scale),
                            pk_bf16(cur.dbv[2] * keep_scale, cur.dbv[3] * keep_scale));
    // x of this lane's window for the A operand: x[w0 + l15][t0 + 4q + i], i < TG + 3
    const int wa = w0 + l15;
    float xa[TG + 3];
#pragma unroll
    for (int i = 0; i < TG + 3; ++i) xa[i] = (wa < B && t0 + 4 * q + i < L) ? cur.xa[i] : 0.f;
    // x of the four windows w0 + 4q + jj at sample t + l15 for the dWc B operand
    float xb[TG][4];
#pragma unroll
    for (int tt = 0; tt < TG; ++tt)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int wb = w0 + 4 * q + jj, s = t0 + tt + l15;
        xb[tt][jj] = (kx && wb < B && s < L) ? cur.xb[tt][jj] : kone;
      }
    // dWc += dP^T X over BOTH steps in one double-rate 16x16x32 MFMA per block: the K slots of
    // lane group q are (step 0, windows 4q .. 4q+3) then (step 1, the same windows) — exactly
    // the dP values and X samples the lane holds after each step (7 MFMAs per group saved)
    static_assert(TG == 2, "dWc pairs the workgroup's two steps into one K = 32 product");
    unsigned dpk[TG][NFB][2], xbp[TG][2];
#pragma unroll
    for (int tt = 0; tt < TG; ++tt) {
      const int t = t0 + tt;
      if (t >= T) {  // (odd T: the pair's second step is absent; zeros contribute nothing)
#pragma unroll
        for (int b = 0; b < NFB; ++b) dpk[tt][b][0] = dpk[tt][b][1] = 0u;
        xbp[tt][0] = xbp[tt][1] = 0u;
        continue;
      }
      const bf16x4 xA = ks.apply(pk_bf16(xa[tt], xa[tt + 1]), pk_bf16(xa[tt + 2], xa[tt + 3]));
      xbp[tt][0] = pk_bf16(xb[tt][0], xb[tt][1]);
      xbp[tt][1] = pk_bf16(xb[tt][2], xb[tt][3]);
      // dropout: the lane holds windows 4q + r of filter column 16b + l15, keep bit 2b + hb0 of
      // window r's hash word. The inverted words of windows (0, 1) and (2, 3) are packed so the
      // bit of block b sits at 2b (first window) and 2b + 16 (second): one shift per block puts
      // both into a packed pair's sign bits (drop_pk), as in the forward
      unsigned pm[2] = {0u, 0u};
      if constexpr (DROP) {
        // the 4 words this lane needs (windows 4q + r, key hq = l15 >> 2) are exactly the ones
        // its quad (lanes 4 hq + 0..3 of row q) computes, one each: ONE hash per lane and a DPP
        // quad broadcast per window instead of four hashes (two quarter-rate multiplies each)
        const unsigned own = cnn_mask_word(smix, w0 + 4 * q + (l15 & 3), t, T, hq);
        const unsigned mi[4] = {~(unsigned)__builtin_amdgcn_mov_dpp((int)own, 0x00, 0xF, 0xF, false) >> hb0,
                                ~(unsigned)__builtin_amdgcn_mov_dpp((int)own, 0x55, 0xF, 0xF, false) >> hb0,
                                ~(unsigned)__builtin_amdgcn_mov_dpp((int)own, 0xAA, 0xF, 0xF, false) >> hb0,
                                ~(unsigned)__builtin_amdgcn_mov_dpp((int)own, 0xFF, 0xF, 0xF, false) >> hb0};
#pragma unroll
        for (int h = 0; h < 2; ++h) pm[h] = (mi[2 * h] & 0xFFFFu) | (mi[2 * h + 1] << 16);
      }
#pragma unroll
      for (int b = 0; b < NFB; ++b) {
        const f32x4 p = mfma16(xA, wc[b], f32x4{0.f, 0.f, 0.f, 0.f});       // [w = 4q + r][f = 16b + l15]
        const f32x4 dA = mfma16(doA, wdb[tt][b], f32x4{0.f, 0.f, 0.f, 0.f});  // same layout
        // act = ReLU + dropout on packed pairs; dP = dAct where act != 0 (kept and p > 0): the
        // packed bf16 dAct times min(act, 1) as int16 lanes (x 1 keeps the bits, x 0 clears)
        unsigned a[2], dp[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          unsigned v = pk_bf16(p[2 * h], p[2 * h + 1]);
          if constexpr (DROP) v = drop_pk(v, pm[h], 2 * b);
          a[h] = relu_pk(v);
          // (inline asm: the compiler rewrote the min / multiply into 6 compares and selects).
          // dp becomes an MFMA operand, and hipcc pads nothing after an asm string: the
          // VALU-write -> MFMA-operand wait states are the s_nop before the paired dWc MFMAs
          // below (round 5 before the pairing: an s_nop 1 in every multiply; without any the
          // MFMA read stale dp on some blocks: NaN conv-weight gradients)
          unsigned one, d = pk_bf16(dA[2 * h], dA[2 * h + 1]);
          asm("v_pk_min_u16 %0, %1, %2" : "=v"(one) : "v"(a[h]), "s"(0x00010001u));
          asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(dp[h]) : "v"(d), "v"(one));
        }
        // act^T as the A operand: A[f = l15][w = 4q + jj]
        acc_wd[tt][b] = mfma16(frag(a[0], a[1]), doB, acc_wd[tt][b]);
        dpk[tt][b][0] = dp[0];
        dpk[tt][b][1] = dp[1];
      }
    }
    // every multiply above stays above (no scheduling across), then the wait states
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 1");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < NFB; ++b)
      acc_wc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag8(dpk[0][b][0], dpk[0][b][1], dpk[1][b][0], dpk[1][b][1]),
                                                          frag8(xbp[0][0], xbp[0][1], xbp[1][0], xbp[1][1]), acc_wc[b], 0, 0, 0);
  };
  const int gs = g_begin + wid;
  if (gs < g_end) {
#pragma unroll
    for (int k = 0; k < NSLOT - 1; ++k) issue(min(gs + k * CNN_NW, g_end - 1), k);
  }
  int slot = 0;
  for (int g = gs; g < g_end; g += CNN_NW) {
    // slot (slot - 1) mod NSLOT was read by the previous group (its values are in registers)
    asm volatile("" ::: "memory");
    issue(min(g + (NSLOT - 1) * CNN_NW, g_end - 1), slot == 0 ? NSLOT - 1 : slot - 1);  // (past the end: never read)
    wait_vmcnt<6 * (NSLOT - 1)>();  // this group's 6 pieces landed (the newer groups' may be in flight)
    GroupLoads cur;
    read_group(slot, cur);
    process(cur, g);
    slot = slot == NSLOT - 1 ? 0 : slot + 1;
  }
  wait_vmcnt<0>();  // the ring aliases `red`: every wave's pieces land before anyone writes it
  __syncthreads();
  // workgroup sums through LDS, one partial per workgroup (fragment layout: lane = 16q + col)
#pragma unroll
  for (int tt = 0; tt < TG; ++tt)
#pragma unroll
    for (int b = 0; b < NFB; ++b) red[((wid * TG + tt) * NFB + b) * 64 + lane] = acc_wd[tt][b];
  __syncthreads();
  for (int e = threadIdx.x; e < TG * NFB * 64; e += 512) {
    f32x4 s = red[e];
#pragma unroll
    for (int k = 1; k < CNN_NW; ++k) s += red[k * TG * NFB * 64 + e];
    const int tt = e / (NFB * 64), rest = e % (NFB * 64);
    if (t0 + tt < T)
      reinterpret_cast<f32x4*>(part_wd)[((size_t)ch * T + t0 + tt) * NFB * 64 + rest] = s;
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < NFB; ++b) red[(wid * NFB + b) * 64 + lane] = acc_wc[b];
  __syncthreads();
  for (int e = threadIdx.x; e < NFB * 64; e += 512) {
    f32x4 s = red[e];
#pragma unroll
    for (int k = 1; k < CNN_NW; ++k) s += red[k * NFB * 64 + e];
    reinterpret_cast<f32x4*>(part_wc)[(size_t)blockIdx.x * NFB * 64 + e] = s;
  }
}

// ------------------------------------------------------------------------------- reduce
// Sums the partials into the flat gradient (+=): blocks [0, nwd) the dense weights (one
// thread per element, nch partials each), [nwd, nwd + nwc) the conv weights + bias (16
// outputs per block, 16 thread groups over the workgroup partials), the last block the dense
// bias, the loss, and the dropout step counter.
__global__ __launch_bounds__(256) void cnn_reduce_kernel(
    const float* __restrict__ part_wd, const float* __restrict__ part_wc, const float* __restrict__ part_f,
    int nch, int nwgb, int nwgf, int T, int Fp, int NFB, int O, int taps, int Kc, int nwd, int nwc,
    float* __restrict__ gWc, float* __restrict__ gWd, float* __restrict__ gbd, float* __restrict__ loss_sum,
    long long* __restrict__ rng) {
  const int bid = blockIdx.x;
  if (bid < nwd) {
    const int i = bid * 256 + threadIdx.x;  // (j, t, f), f fastest
    const int nf = T * Fp;
    if (i >= O * nf) return;
    const int j = i / nf, rest = i % nf, t = rest / Fp, f = rest % Fp;
    const int b = f >> 4, lanep = ((f & 15) >> 2) * 16 + j, r = f & 3;
    const size_t stride = (size_t)T * NFB * 64 * 4;
    const float* p = part_wd + (((size_t)t * NFB + b) * 64 + lanep) * 4 + r;
    // 16 independent loads per latency round (one round at the 14 chunks of 256 CUs; was one
    // round per 4 chunks): past the end they re-load the last chunk and are dropped
    float s4[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nch; c += 16) {
      float v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = p[(size_t)min(c + k, nch - 1) * stride];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (c + k < nch) s4[k & 3] += v[k];
    }
    gWd[(size_t)j * nf + rest] += (s4[0] + s4[1]) + (s4[2] + s4[3]);
    return;
  }
  if (bid < nwd + nwc) {
    __shared__ float sh[16][17];
    const int o = (bid - nwd) * 16 + (threadIdx.x & 15), grp = threadIdx.x >> 4;  // o = f * 16 + kk
    const int f = o >> 4, kk = o & 15;
    float s = 0.f;
    if (f < Fp && kk <= taps) {
      const int b = f >> 4, lanep = ((f & 15) >> 2) * 16 + kk, r = f & 3;
      const float* p = part_wc + (((size_t)b * 64 + lanep) * 4 + r);
      const size_t stride = (size_t)NFB * 64 * 4;
      // 16 independent loads per round, as above (one round at 252 workgroup partials)
      float s4[4] = {0.f, 0.f, 0.f, 0.f};
      for (int c = grp; c < nwgb; c += 256) {
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = p[(size_t)min(c + 16 * k, nwgb - 1) * stride];
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (c + 16 * k < nwgb) s4[k & 3] += v[k];
      }
      s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    }
    sh[grp][threadIdx.x & 15] = s;
    __syncthreads();
    if (grp == 0 && f < Fp && kk <= taps) {
      float tsum = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) tsum += sh[k][threadIdx.x & 15];
      gWc[(size_t)f * Kc + kk] += tsum;
    }
    return;
  }
  // dense bias, loss, step counter: thread c loads forward workgroup c's 17 partials (one
  // latency round; the serial 256-load chain per output took 63 us), LDS columns summed by 17
  // threads
  __shared__ float pf[17][257];
  {
    float v[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) v[k] = 0.f;
    for (int c = threadIdx.x; c < nwgf; c += 256)
#pragma unroll
      for (int k = 0; k < 17; ++k) v[k] += part_f[c * 32 + k];
#pragma unroll
    for (int k = 0; k < 17; ++k) pf[k][threadIdx.x] = v[k];
  }
  __syncthreads();
  // 15 threads per column (255 of 256) sum every 15th entry, then 17 threads the 15 sums (the
  // 17-thread pass over 256 entries each was a 64-deep chain of LDS reads)
  __shared__ float pf2[17][16];
  if (threadIdx.x < 255) {
    const int k = threadIdx.x / 15, part = threadIdx.x % 15;
    float sp = 0.f;
    for (int c = part; c < 256; c += 15) sp += pf[k][c];
    pf2[k][part] = sp;
  }
  __syncthreads();
  if (threadIdx.x < 17) {
    float s = 0.f;
#pragma unroll
    for (int part = 0; part < 15; ++part) s += pf2[threadIdx.x][part];
    if (threadIdx.x < 16) {
      if (threadIdx.x < O) gbd[threadIdx.x] += s;
    } else if (loss_sum != nullptr) {
      loss_sum[0] += s;
    }
  }
  if (threadIdx.x == 0 && rng != nullptr) rng[0] += 1;
}

// --------------------------------------------------------------------------------- pack
// fp32 flat parameters -> the bf16 operand images: WcA [Fp][Kc] (a plain cast, the bias in
// column taps), WdF (forward A fragments: lane (j = l15, q) holds Wd[j][t Fp + 16b + 4q + jj])
// and WdB (backward B fragments: lane (f = l15, q) holds Wd[4q + jj][t Fp + 16b + f]), both
// [T][NFB][64 lanes][4] — rows j >= O are zero.
__global__ __launch_bounds__(256) void cnn_pack_kernel(const float* __restrict__ Wc, const float* __restrict__ Wd,
                                                       int T, int Fp, int NFB, int Kc, int O, bf16_t* __restrict__ WcA,
                                                       bf16_t* __restrict__ WdF, bf16_t* __restrict__ WdB) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int nfr = T * NFB * 64;
  const long nf = (long)T * Fp;
  if (i < nfr) {
    // WdB (8-B unit i): [T][NFB][64 lanes][4]; WdF: per step 3 block pairs of [64 lanes][8]
    // (block 2p in the lane's first 8 B, 2p+1 in the next) then block 6 [64 lanes][4]
    const int lane = i & 63, tb = i >> 6, t = tb / NFB, b = tb % NFB;
    const int l15 = lane & 15, q = lane >> 4;
    const int e = i % (NFB * 64);  // 8-B unit within step t of the WdF image
    const int bf = e < 384 ? 2 * (e / 128) + (e & 1) : 6, lf = e < 384 ? (e % 128) >> 1 : e - 384;
    unsigned short vf[4], vb[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = lf & 15, f = 16 * bf + 4 * (lf >> 4) + jj;
      vf[jj] = j < O ? f2bf(Wd[(long)j * nf + (long)t * Fp + f]) : 0;
      const int j2 = 4 * q + jj, f2 = 16 * b + l15;
      vb[jj] = j2 < O ? f2bf(Wd[(long)j2 * nf + (long)t * Fp + f2]) : 0;
    }
    *reinterpret_cast<uint2*>(WdF + (size_t)i * 4) = uint2{vf[0] | ((unsigned)vf[1] << 16), vf[2] | ((unsigned)vf[3] << 16)};
    *reinterpret_cast<uint2*>(WdB + (size_t)i * 4) = uint2{vb[0] | ((unsigned)vb[1] << 16), vb[2] | ((unsigned)vb[3] << 16)};
  } else if (i < nfr + Fp * Kc) {
    const int k = i - nfr;
    WcA[k] = f2bf(Wc[k]);
  }
}

// ------------------------------------------------------------------------ SGD + pack
// Keras SGD (elementwise.hip sgd_dev_kernel: device iteration counter, Nesterov) over the flat
// parameters [Wc Fp x Kc | Wd 16 x T Fp | bd] AND, in the same pass, the bf16 operand images
// cnn_pack_kernel would write next (WcA, WdF, WdB): one launch per update instead of two
// (round 5). Each updated weight is scattered to its image positions (the inverse of the pack
// kernel's gather); rows j >= O of the dense block are padding and stay zero.
__global__ __launch_bounds__(256) void cnn_sgd_pack_kernel(float* __restrict__ p, float* __restrict__ g,
                                                           float* __restrict__ vel, long n, float* __restrict__ step,
                                                           float lr, float decay, float momentum, int nesterov,
                                                           float gscale, int zero_g, int T, int Fp, int NFB, int Kc,
                                                           int O, bf16_t* __restrict__ WcA, bf16_t* __restrict__ WdF,
                                                           bf16_t* __restrict__ WdB) {
  const float it = step[0];
  const float lr_t = lr / (1.f + decay * it);
  const long nc = (long)Fp * Kc, nf = (long)T * Fp, nd = 16 * nf;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gi = g[i] * gscale;
    const float v = momentum * vel[i] - lr_t * gi;
    vel[i] = v;
    const float pn = p[i] + (nesterov ? (momentum * v - lr_t * gi) : v);
    p[i] = pn;
    if (zero_g) g[i] = 0.f;
    if (i < nc) {
      WcA[i] = f2bf(pn);
    } else if (i < nc + nd) {
      const long e = i - nc;
      const int j = (int)(e / nf), rest = (int)(e % nf), t = rest / Fp, f = rest % Fp;
      const unsigned short h = j < O ? f2bf(pn) : 0;
      const int b = f >> 4, l15 = f & 15;
      // WdB: lane 16 (j >> 2) + (f & 15) of block b, element j & 3
      WdB[(((size_t)t * NFB + b) * 64 + 16 * (j >> 2) + l15) * 4 + (j & 3)] = h;
      // WdF: lf = 16 q + j (q = (f & 15) >> 2); pairs of blocks (2p, 2p + 1) interleave per lane
      const int lf = 16 * (l15 >> 2) + j;
      const int eu = b < 6 ? 128 * (b >> 1) + 2 * lf + (b & 1) : 384 + lf;
      WdF[((size_t)t * NFB * 64 + eu) * 4 + (f & 3)] = h;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* ticket = reinterpret_cast<unsigned*>(step + 1);
    if (atomicAdd(ticket, 1u) == gridDim.x - 1) {
      step[0] = it + 1.f;
      *ticket = 0u;
    }
  }
}

// -------------------------------------------------------------------------------- launch
bool cnn_fused_supported(const CnnDims& d) {
  return d.C == 1 && d.T == CNN_T && (d.Fp >> 4) == CNN_NFB && d.Fp % 16 == 0 && d.taps <= 15 && d.Kc == 16 &&
         d.O >= 1 && d.O <= 16 && d.L % 4 == 0 && d.L == d.T + d.taps - 1 && (d.drop_p == 0.f || d.drop_p == 0.5f);
}

int cnn_fwd_grid(int B) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    return n;
  }();
  const int ngroups = (B + 15) / 16;
  return std::max(1, std::min(cus, (ngroups + CNN_NW - 1) / CNN_NW));
}

int cnn_bwd_chunks(int B) {
  const int ntg = (CNN_T + CNN_TG - 1) / CNN_TG;
  const int ngroups = (B + 15) / 16;
  const int cus = cnn_fwd_grid(1 << 30);  // the CU count
  return std::max(1, std::min(std::max(1, cus / ntg), (ngroups + CNN_NW - 1) / CNN_NW));
}

void launch_cnn_pack(const float* Wc, const float* Wd, const CnnDims& d, bf16_t* WcA, bf16_t* WdF, bf16_t* WdB,
                     hipStream_t s) {
  const int n = d.T * (d.Fp / 16) * 64 + d.Fp * d.Kc;
  hipLaunchKernelGGL(cnn_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, s, Wc, Wd, d.T, d.Fp, d.Fp / 16, d.Kc,
                     d.O, WcA, WdF, WdB);
}

void launch_cnn_sgd_pack(float* p, float* g, float* vel, long n, float* step, float lr, float decay, float momentum,
                         int nesterov, float gscale, int zero_g, const CnnDims& d, bf16_t* WcA, bf16_t* WdF,
                         bf16_t* WdB, hipStream_t s) {
  long b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(cnn_sgd_pack_kernel, dim3((int)b), dim3(256), 0, s, p, g, vel, n, step, lr, decay, momentum,
                     nesterov, gscale, zero_g, d.T, d.Fp, d.Fp / 16, d.Kc, d.O, WcA, WdF, WdB);
}

void launch_cnn_forward(const float* x, int B, const CnnDims& d, const bf16_t* WcA, const bf16_t* WdF,
                        const float* bd, const float* y, float* dout, float* pred, float* part, int train,
                        int loss_kind, float clip, float scale, unsigned seed, const long long* rng, hipStream_t s) {
  const int grid = cnn_fwd_grid(B);
  const int drop = (train && d.drop_p > 0.f) ? 1 : 0;
  const float keep_scale = drop ? 1.f / (1.f - d.drop_p) : 1.f;
  if (train && drop)
    hipLaunchKernelGGL((cnn_fwd_kernel<CNN_NFB, CNN_T, true, true>), dim3(grid), dim3(512), 0, s, x, B, d.L, WcA,
                       d.Kc, reinterpret_cast<const bf16x4*>(WdF), bd, d.O, y, dout, pred, part, d.taps, loss_kind,
                       clip, scale, keep_scale, drop, seed, rng, 0);
  else if (train)
    hipLaunchKernelGGL((cnn_fwd_kernel<CNN_NFB, CNN_T, true, false>), dim3(grid), dim3(512), 0, s, x, B, d.L, WcA,
                       d.Kc, reinterpret_cast<const bf16x4*>(WdF), bd, d.O, y, dout, pred, part, d.taps, loss_kind,
                       clip, scale, keep_scale, 0, seed, rng, 0);
  else
    hipLaunchKernelGGL((cnn_fwd_kernel<CNN_NFB, CNN_T, false, false>), dim3(grid), dim3(512), 0, s, x, B, d.L, WcA,
                       d.Kc, reinterpret_cast<const bf16x4*>(WdF), bd, d.O, y, dout, pred, part, d.taps, loss_kind,
                       clip, scale, keep_scale, 0, seed, rng, 0);
}

void launch_cnn_backward(const float* x, int B, const CnnDims& d, const bf16_t* WcA, const bf16_t* WdB,
                         const float* dout, unsigned seed, const long long* rng, float* part_wd, float* part_wc,
                         hipStream_t s) {
  const int ntg = (d.T + CNN_TG - 1) / CNN_TG;
  const int nch = cnn_bwd_chunks(B);
  const int drop = d.drop_p > 0.f ? 1 : 0;
  const float keep_scale = drop ? 1.f / (1.f - d.drop_p) : 1.f;
  if (drop)
    hipLaunchKernelGGL((cnn_bwd_kernel<CNN_NFB, CNN_TG, true>), dim3(ntg * nch), dim3(512), 0, s, x, B, d.L, WcA,
                       d.Kc, reinterpret_cast<const bf16x4*>(WdB), dout, d.T, d.taps, keep_scale, drop, seed, rng, nch,
                       part_wd, part_wc, 0);
  else
    hipLaunchKernelGGL((cnn_bwd_kernel<CNN_NFB, CNN_TG, false>), dim3(ntg * nch), dim3(512), 0, s, x, B, d.L, WcA,
                       d.Kc, reinterpret_cast<const bf16x4*>(WdB), dout, d.T, d.taps, keep_scale, drop, seed, rng, nch,
                       part_wd, part_wc, 0);
}

void launch_cnn_reduce(const float* part_wd, const float* part_wc, const float* part_f, int B, const CnnDims& d,
                       float* gWc, float* gWd, float* gbd, float* loss_sum, long long* rng, hipStream_t s) {
  const int nch = cnn_bwd_chunks(B), ntg = (d.T + CNN_TG - 1) / CNN_TG;
  const int nwd = (d.O * d.T * d.Fp + 255) / 256, nwc = d.Fp;  // 16 (f, kk) outputs per block: Fp * 16 / 16
  hipLaunchKernelGGL(cnn_reduce_kernel, dim3(nwd + nwc + 1), dim3(256), 0, s, part_wd, part_wc, part_f, nch,
                     ntg * nch, cnn_fwd_grid(B), d.T, d.Fp, d.Fp / 16, d.O, d.taps, d.Kc, nwd, nwc, gWc, gWd, gbd,
                     loss_sum, rng);
}

long cnn_part_floats(int B, const CnnDims& d, long* wd, long* wc, long* f) {
  const int nch = cnn_bwd_chunks(B), ntg = (d.T + CNN_TG - 1) / CNN_TG;
  *wd = (long)nch * d.T * (d.Fp / 16) * 64 * 4;
  *wc = (long)ntg * nch * (d.Fp / 16) * 64 * 4;
  *f = (long)cnn_fwd_grid(B) * 32;
  return *wd + *wc + *f;
}

}  // namespace wf
