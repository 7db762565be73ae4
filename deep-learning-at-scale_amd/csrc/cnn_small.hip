// wellflow — K consecutive small-batch training steps of the reference CNN (cnn.py:110-118:
// Conv1D(1 -> 100, width 13) + ReLU -> Dropout(0.5) -> Dense(3600 -> 12), clipped MAE, Keras
// SGD-Nesterov) in ONE persistent launch, at the reference's own batch of 20 (cnn.py:128).
// SURVEY.md §2.4 K1-K9; round-5 VERDICT item 3(b).
//
// At 20 windows a step is ~9 MFLOP and the fused path's four launches (forward, backward,
// reduce, SGD + operand pack) cost ~28 us of fixed latency (profiles/r6/job_default/
// cnn_b20_kernel_stats.csv). Here G workgroups each own 4 filters: their conv weights and the
// 12 x 36 x 4 dense weights that read those filters, in fp32 with the SGD velocities, in LDS for
// the whole launch. The model splits so that ONE exchange per step suffices:
//   conv + ReLU + dropout of the own filters (all windows) -> the own filters' share of the 12
//   dense outputs -> publish as {value, tag} granules | poll every worker's share (fixed
//   summation order): prediction, loss, dOut — identical in every worker | dWd, dAct (dropout
//   and ReLU masks), dWc of the own filters, all local | SGD on the own parameters; the dense
//   bias is replicated: every worker applies the same update from the same dOut.
// Computed in fp32 on the VALU (the batch is far too small for MFMA tiles). The granules are
// double-buffered by step parity (a worker is at most one step ahead of any reader: it needs
// every worker's step-k share before it writes its step-(k+1) share); the tag names the launch
// (sync[3], advanced by the last worker out) and the step. Dropout draws the fused kernels' mask
// (cnn_fused.hip, models/cnn.py cnn_dropout_mask) from the engine's device step counter.
// Bounded polls: a lost hand-off sets a sticky error word (results garbage, the host raises).
// Every reduction has a fixed order, so K fused steps equal K single-step launches bit for bit.
#include <type_traits>
#include "common.h"
#include "kernels.h"

namespace wf {

namespace {

constexpr int CS_FPW = 4;     // filters per worker
constexpr int CS_T = 36;      // output steps
constexpr int CS_L = 48;      // window length
constexpr int CS_KC = 16;     // conv K slots (13 taps + bias + 2 zero)
constexpr int CS_FP = 112;    // padded filters of the flat layout
constexpr int CS_OP = 16;     // padded outputs of the flat layout
constexpr int CS_TAPS = CS_L - CS_T + 1;  // 13 (the K slot after the taps is the bias)
constexpr int CS_MAXB = 64;
constexpr int CS_NT = 1024;  // 16 waves: 4 per SIMD hide the LDS latency of the VALU loops
// scratch (floats): share granules [2 parities][28 workers][64 x 16], then the summed outputs
// [2 parities][64 x 16]
constexpr int CS_P1 = 0, CS_P2 = 2 * 28 * 64 * 16 * 2;

typedef __attribute__((address_space(1))) unsigned cs_g32;
typedef unsigned cs_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned cs_lowbias32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(CS_NT, 1) void cnn_small_kernel(const CnnSmallArgs a) {
  const int B = a.B, K = a.K, O = a.O, taps = a.taps;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wk = blockIdx.x, G = gridDim.x;
  const int f0 = CS_FPW * wk;  // first owned filter
  // LDS
  __shared__ __attribute__((aligned(16))) float xs[CS_MAXB][CS_L];
  __shared__ float ysm[CS_MAXB][CS_OP];
  // [.][filter][step]: steps fastest, so lanes over consecutive steps hit consecutive banks in
  // every loop below ([.][step][filter] put the dWc loop into 16-way bank conflicts)
  __shared__ __attribute__((aligned(16))) float act[CS_MAXB][CS_FPW][CS_T];  // relu(P) kept (unscaled)
  __shared__ __attribute__((aligned(16))) float dp[CS_MAXB][CS_FPW][CS_T];   // dAct -> dP (masked)
  __shared__ __attribute__((aligned(16))) float dout[CS_MAXB][CS_OP];
  __shared__ __attribute__((aligned(16))) float wc[CS_FPW][CS_KC];
  __shared__ float vc[CS_FPW][CS_KC];
  __shared__ __attribute__((aligned(16))) float wd[CS_OP][CS_FPW][CS_T];
  __shared__ float vd[CS_OP][CS_FPW][CS_T];
  __shared__ float bd[CS_OP], vb[CS_OP];
  __shared__ __attribute__((aligned(16))) float gwc[CS_FPW][CS_TAPS + 1][CS_T];  // dWc partials per output step
  __shared__ float lred[CS_NT / 64];
  __shared__ __attribute__((aligned(16))) float red2[48][28];  // hop 1 of the output sums: [own output][share]
  __shared__ unsigned sflag;
  __shared__ __attribute__((aligned(16))) unsigned hw[CS_MAXB * CS_T];  // the step's dropout hash words

  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.scr, 0, 0x7FFFFFFF, 0x00020000);
  auto st8 = [&](unsigned val, unsigned tag, int fo) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0)),
                                                             (cs_u32x2{val, tag})), rs, fo * 4, 0, 16);
  };
  auto ld8 = [&](int fo) { return __builtin_bit_cast(cs_u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, fo * 4, 0, 16)); };

  // ---- owned parameters and velocities (flat layout: Wc [112][16] | Wd [16][36 * 112] | bd [16])
  const long oWd = (long)CS_FP * CS_KC, obd = oWd + (long)CS_OP * CS_T * CS_FP;
  for (int i = tid; i < CS_FPW * CS_KC; i += CS_NT) {
    const int fl = i / CS_KC, kk = i % CS_KC;
    const long e = (long)(f0 + fl) * CS_KC + kk;
    wc[fl][kk] = a.p[e];
    vc[fl][kk] = a.vel[e];
  }
  for (int i = tid; i < CS_OP * CS_T * CS_FPW; i += CS_NT) {
    const int j = i / (CS_T * CS_FPW), fl = (i / CS_T) % CS_FPW, t = i % CS_T;
    const long e = oWd + (long)j * CS_T * CS_FP + t * CS_FP + f0 + fl;
    wd[j][fl][t] = a.p[e];
    vd[j][fl][t] = a.vel[e];
  }
  if (tid < CS_OP) {
    bd[tid] = a.p[obd + tid];
    vb[tid] = a.vel[obd + tid];
  }
  if (tid == 0) sflag = 0u;
  const float it0 = a.step[0];
  const unsigned rng0 = (unsigned)a.rng[0];
  const unsigned lc = __hip_atomic_load((cs_g32*)(a.sync + 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float ks = a.keep_scale;

  // ---- batch prefetch (row ids one step ahead): piece i = tid + 256 q of the [B][48] x tile and
  // [B][O] y tile
  constexpr int NXP = CS_MAXB * CS_L / CS_NT;   // 3
  constexpr int NYP = CS_MAXB * CS_OP / CS_NT;  // 1
  float xv[NXP], yv[NYP];
  long xid[NXP], yid[NYP];
  auto fetch_ids = [&](int k) {
#pragma unroll
    for (int q = 0; q < NXP; ++q) {
      const int w = (tid + CS_NT * q) / CS_L;
      xid[q] = (w < B && k < K) ? (long)(a.rows != nullptr ? a.rows[(long)k * B + w] : (long)k * B + w) : 0;
    }
#pragma unroll
    for (int q = 0; q < NYP; ++q) {
      const int w = (tid + CS_NT * q) / CS_OP;
      yid[q] = (w < B && k < K) ? (long)(a.rows != nullptr ? a.rows[(long)k * B + w] : (long)k * B + w) : 0;
    }
  };
  auto prefetch = [&]() {
#pragma unroll
    for (int q = 0; q < NXP; ++q) {
      const int i = tid + CS_NT * q, w = i / CS_L, s = i % CS_L;
      long r = xid[q];
      r = r < 0 ? 0 : (r >= a.nrows ? a.nrows - 1 : r);
      xv[q] = w < B ? a.X[r * CS_L + s] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < NYP; ++q) {
      const int i = tid + CS_NT * q, w = i / CS_OP, j = i % CS_OP;
      long r = yid[q];
      r = r < 0 ? 0 : (r >= a.nrows ? a.nrows - 1 : r);
      yv[q] = (w < B && j < O) ? a.Y[r * O + j] : 0.f;
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int q = 0; q < NXP; ++q) {
      const int i = tid + CS_NT * q;
      xs[i / CS_L][i % CS_L] = xv[q];
    }
#pragma unroll
    for (int q = 0; q < NYP; ++q) {
      const int i = tid + CS_NT * q;
      ysm[i / CS_OP][i % CS_OP] = yv[q];
    }
  };
  fetch_ids(0);
  prefetch();
  fetch_ids(1);
  for (int i = tid; i < 48 * 28; i += CS_NT) (&red2[0][0])[i] = 0.f;
  __syncthreads();

  unsigned gspins = 0;
  int kcur = 0;
  auto stamp = [&](int ph) {  // diagnostics: phase boundaries of the first 64 steps
    if (a.stamps != nullptr && tid == 0 && kcur < 64)
      a.stamps[((size_t)wk * 64 + kcur) * 16 + ph] = __builtin_amdgcn_s_memrealtime();
  };
  for (int k = 0; k < K; ++k) {
    const int par = k & 1;
    const unsigned tag = (lc << 12) + (unsigned)k + 1u;
    kcur = k;
    stamp(0);
    stage();
    // the dropout hash of every (window, step), staged beside x: the fused kernels' mask word
    // (cnn_fused.hip cnn_mask_word) depends on the filter only through the bit it selects, and
    // a worker's 4 filters share the word's other inputs (q = f >> 2 & 3 = wk & 3), so one hash
    // per (window, step) serves all 4 (the conv computed it 4 times per element before)
    const unsigned rstep = rng0 + (unsigned)k;
    const unsigned smix = cs_lowbias32(a.seed ^ cs_lowbias32(rstep + 0x9E3779B9u));
    if (a.drop) {
      for (int i = tid; i < B * CS_T; i += CS_NT) hw[i] = cs_lowbias32(((unsigned)i * 4u + (unsigned)(wk & 3)) ^ smix);
    }
    __syncthreads();
    stamp(1);
    if (k + 1 < K) {
      prefetch();
      fetch_ids(k + 2);
    }
    // ---- conv + ReLU + dropout of the own filters, every window and step
    // (every loop below has compile-time trip counts and is unrolled: the runtime-bounded forms
    // were LDS-latency chains, one load -> wait -> fma per iteration: conv 9.3 us per step)
    // task (window, filter, 4 steps): x[t4 .. t4 + 15] and the filter row in 8 float4 reads
    for (int i = tid; i < B * CS_FPW * (CS_T / 4); i += CS_NT) {
      const int w = i / (CS_FPW * (CS_T / 4)), fl = (i / (CS_T / 4)) % CS_FPW, t4 = 4 * (i % (CS_T / 4));
      float wcr[CS_KC], xw[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        *reinterpret_cast<float4*>(&wcr[4 * c]) = *reinterpret_cast<const float4*>(&wc[fl][4 * c]);
        *reinterpret_cast<float4*>(&xw[4 * c]) = *reinterpret_cast<const float4*>(&xs[w][t4 + 4 * c]);
      }
      float pv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pv[e] = wcr[CS_TAPS];  // the conv bias (K slot = taps)
#pragma unroll
        for (int kk = 0; kk < CS_TAPS; ++kk) pv[e] = fmaf(wcr[kk], xw[e + kk], pv[e]);
      }
      uint4 mw = make_uint4(~0u, ~0u, ~0u, ~0u);  // the 4 steps' hash words (all-keep without dropout)
      if (a.drop) mw = *reinterpret_cast<const uint4*>(&hw[w * CS_T + t4]);
      const int f = f0 + fl, r = f & 3, bsh = 2 * (f >> 4) + (r >> 1) + 16 * (r & 1);
      const float o0 = ((mw.x >> bsh) & 1u) != 0u && pv[0] > 0.f ? pv[0] : 0.f;
      const float o1 = ((mw.y >> bsh) & 1u) != 0u && pv[1] > 0.f ? pv[1] : 0.f;
      const float o2 = ((mw.z >> bsh) & 1u) != 0u && pv[2] > 0.f ? pv[2] : 0.f;
      const float o3 = ((mw.w >> bsh) & 1u) != 0u && pv[3] > 0.f ? pv[3] : 0.f;
      *reinterpret_cast<float4*>(&act[w][fl][t4]) = make_float4(o0, o1, o2, o3);
    }
    __syncthreads();
    stamp(2);
    // ---- this worker's share of the dense outputs -> granules (parity par)
    // (vectorised over 4 consecutive steps in every loop below: float4 LDS reads, 4 outputs per
    // task; each phase was LDS-instruction bound at one element per task)
    // four lanes per (window, output), one filter each, combined by two xor shuffles
    for (int i0 = 0; i0 < 4 * B * O; i0 += CS_NT) {
      const int i = i0 + tid;
      const bool act_i = i < 4 * B * O;
      const int pr = act_i ? i >> 2 : 0, fl = i & 3, w = pr / O, j = pr % O;
      float s = 0.f;
#pragma unroll
      for (int t4 = 0; t4 < CS_T; t4 += 4) {
        const float4 wv = *reinterpret_cast<const float4*>(&wd[j][fl][t4]);
        const float4 av = *reinterpret_cast<const float4*>(&act[w][fl][t4]);
        s = fmaf(wv.x, av.x, s);
        s = fmaf(wv.y, av.y, s);
        s = fmaf(wv.z, av.z, s);
        s = fmaf(wv.w, av.w, s);
      }
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      if (act_i && fl == 0) st8(__float_as_uint(s), tag, CS_P1 + ((par * G + wk) * CS_MAXB * CS_OP + w * CS_OP + j) * 2);
    }
    stamp(3);
    // ---- the shares are summed in two hops (one 25-way read of every output per worker moved
    // 48 KiB per worker per poll round: 9.4 us; watching one granule per producer, then reading
    // all shares once: 5.4 us, the bulk read alone 3.5): worker wk sums outputs o = wk + G l over
    // the G shares (fixed order) and publishes them; then every worker reads the B x O sums
    auto poll_more = [&](bool ok) {
      if (__builtin_amdgcn_ballot_w64(!ok) == 0ull || sflag != 0u) return false;
      if ((++gspins & 63u) == 0u &&
          __hip_atomic_load((cs_g32*)(a.sync + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        if (lane == 0) sflag = 1u;
        return false;
      }
      if (gspins > a.spin_limit) {
        __hip_atomic_store((cs_g32*)(a.sync + 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0) sflag = 1u;
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
      return true;
    };
    const int nout = B * O, nl = wk < nout ? (nout - wk + G - 1) / G : 0;
    for (int i0 = 0; i0 < nl * G; i0 += CS_NT) {
      const int i = i0 + tid;
      const bool act_i = i < nl * G;
      const int l = act_i ? i / G : 0, g = act_i ? i % G : 0;
      const int o = wk + G * l;
      float v = 0.f;
      bool more = true;
      while (more) {
        bool ok = true;
        if (act_i) {
          const cs_u32x2 u = ld8(CS_P1 + ((par * G + g) * CS_MAXB * CS_OP + (o / O) * CS_OP + (o % O)) * 2);
          v = __uint_as_float(u[0]);
          ok = u[1] == tag;
        }
        more = poll_more(ok);
      }
      if (act_i) red2[l][g] = v;
    }
    __syncthreads();
    for (int l = tid; l < nl; l += CS_NT) {
      float sum = 0.f;
      // shares g >= G stay zero (cleared at launch start): 7 float4 reads, one add chain in share
      // order (a runtime-bounded loop was 25 dependent LDS round trips, ~0.6 us)
#pragma unroll
      for (int c = 0; c < 7; ++c) {
        const float4 v = *reinterpret_cast<const float4*>(&red2[l][4 * c]);
        sum += v.x;
        sum += v.y;
        sum += v.z;
        sum += v.w;
      }
      st8(__float_as_uint(sum), tag, CS_P2 + (par * CS_MAXB * CS_OP + wk + G * l) * 2);
    }
    stamp(9);
    // ---- every output: prediction, loss, dOut
    float lsum = 0.f;
    for (int i0 = 0; i0 < nout; i0 += CS_NT) {
      const int i = i0 + tid;
      const bool act_i = i < nout;
      const int w = act_i ? i / O : 0, j = act_i ? i % O : 0;
      float s = 0.f;
      bool more = true;
      while (more) {
        bool ok = true;
        if (act_i) {
          const cs_u32x2 u = ld8(CS_P2 + (par * CS_MAXB * CS_OP + i) * 2);
          s = __uint_as_float(u[0]);
          ok = u[1] == tag;
        }
        more = poll_more(ok);
      }
      if (act_i) {
        const float pv = s * ks + bd[j], yvv = ysm[w][j];
        float l, dd;
        if (a.loss_kind == 0) {
          const float e = pv - yvv;
          l = e * e;
          dd = 2.f * e;
        } else {
          const float e = yvv - pv, ae = fabsf(e);
          l = fminf(ae, a.clip);
          const float sg = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f);
          dd = ae <= a.clip ? -sg : 0.f;
        }
        lsum += l;
        dout[w][j] = dd * a.scale;
      }
    }
    stamp(10);
    if (wk == 0) {
      const float ls = block_sum<CS_NT>(lsum, lred);
      if (tid == 0 && a.loss_acc != nullptr) atomicAdd(a.loss_acc, ls);
    } else {
      __syncthreads();
    }
    stamp(4);
    // ---- dWd (own columns) = ks * dOut^T act, and dAct = ks * dOut Wd masked -> dP
    // task (j, fl, 4 steps), tid < CS_OP * CS_FPW * CS_T / 4 = 576: the SGD below updates the
    // same 4 parameters in the same thread
    constexpr int NWD = CS_OP * CS_FPW * (CS_T / 4);
    float4 gwd = make_float4(0.f, 0.f, 0.f, 0.f);
    const int dj = tid / (CS_FPW * (CS_T / 4)), dfl = (tid / (CS_T / 4)) % CS_FPW, dt4 = 4 * (tid % (CS_T / 4));
    if (tid < NWD && dj < O) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int w0 = 0; w0 < B; w0 += 4) {  // B % 4 == 0 (launcher)
#pragma unroll
        for (int w = w0; w < w0 + 4; ++w) {
          const float d = dout[w][dj];
          const float4 av = *reinterpret_cast<const float4*>(&act[w][dfl][dt4]);
          s.x = fmaf(d, av.x, s.x);
          s.y = fmaf(d, av.y, s.y);
          s.z = fmaf(d, av.z, s.z);
          s.w = fmaf(d, av.w, s.w);
        }
      }
      gwd = make_float4(ks * s.x, ks * s.y, ks * s.z, ks * s.w);
    }
    // (no barrier: dAct writes dP to its own buffer, so it runs beside dWd's reads of act)
    stamp(5);
    for (int i = tid; i < B * CS_FPW * (CS_T / 4); i += CS_NT) {
      const int w = i / (CS_FPW * (CS_T / 4)), fl = (i / (CS_T / 4)) % CS_FPW, t4 = 4 * (i % (CS_T / 4));
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      float dr[CS_OP];  // the window's dOut row in 4 float4 reads (was 12 scalar reads)
#pragma unroll
      for (int c = 0; c < CS_OP / 4; ++c)
        *reinterpret_cast<float4*>(&dr[4 * c]) = *reinterpret_cast<const float4*>(&dout[w][4 * c]);
#pragma unroll
      for (int j = 0; j < CS_OP; ++j)
        if (j < O) {
          const float d = dr[j];
          const float4 wv = *reinterpret_cast<const float4*>(&wd[j][fl][t4]);
          s.x = fmaf(d, wv.x, s.x);
          s.y = fmaf(d, wv.y, s.y);
          s.z = fmaf(d, wv.z, s.z);
          s.w = fmaf(d, wv.w, s.w);
        }
      const float4 av = *reinterpret_cast<const float4*>(&act[w][fl][t4]);
      *reinterpret_cast<float4*>(&dp[w][fl][t4]) =
          make_float4(av.x > 0.f ? ks * s.x : 0.f, av.y > 0.f ? ks * s.y : 0.f, av.z > 0.f ? ks * s.z : 0.f,
                      av.w > 0.f ? ks * s.w : 0.f);
    }
    __syncthreads();
    stamp(6);
    // dWc[fl][kk] = sum_{t, w} dP[w][t][fl] x[w][t + kk] (kk = taps: the conv bias, sum dP): task
    // (fl, kk, t) with t fastest sums over the windows (consecutive lanes read consecutive
    // steps: the window-strided form of this loop ran into 16-way bank conflicts, 10 us)
    // task (filter, 4 steps, window class w % 4, tap half): one float4 of dP and three of x give
    // 4 x 7 products per window; the partial for (filter, tap) lands in gwc[fl][kk][4 t4i + wq]
    // (36 partials per parameter, summed in the SGD below)
    // (the tap half is wave-uniform: threads [0, 144) take kk 0..6, threads [192, 336) kk 7..13,
    // so both halves index their x registers with compile-time offsets)
    auto dwc_half = [&](auto khc, int u) {
      constexpr int kh = decltype(khc)::value;
      const int wq = u & 3, t4i = (u >> 2) % (CS_T / 4), fl = u / (4 * (CS_T / 4));
      const int t4 = 4 * t4i;
      float s[7];
#pragma unroll
      for (int q = 0; q < 7; ++q) s[q] = 0.f;
      for (int w = wq; w < B; w += 4) {  // B % 4 == 0 (launcher)
        const float4 av = *reinterpret_cast<const float4*>(&dp[w][fl][t4]);
        const float d[4] = {av.x, av.y, av.z, av.w};
        float xw[12];  // x[t4 + 4 kh + j]
#pragma unroll
        for (int c = 0; c < 3; ++c)
          *reinterpret_cast<float4*>(&xw[4 * c]) = *reinterpret_cast<const float4*>(&xs[w][t4 + 4 * kh + 4 * c]);
#pragma unroll
        for (int q = 0; q < 7; ++q) {
          const int kk = 7 * kh + q;
#pragma unroll
          for (int e = 0; e < 4; ++e) s[q] = fmaf(d[e], kk < CS_TAPS ? xw[e + kk - 4 * kh] : 1.f, s[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < 7; ++q) gwc[fl][7 * kh + q][4 * t4i + wq] = s[q];
    };
    constexpr int NDWC = CS_FPW * (CS_T / 4) * 4;  // 144
    if (tid < NDWC) dwc_half(std::integral_constant<int, 0>{}, tid);
    else if (tid >= 192 && tid < 192 + NDWC) dwc_half(std::integral_constant<int, 1>{}, tid - 192);
    __syncthreads();
    stamp(7);
    // ---- Keras SGD (lr / (1 + decay * iterations), momentum, Nesterov) on the own parameters and
    // the replicated dense bias (same dOut everywhere -> same update everywhere)
    const float it = it0 + (float)k;
    const float lr_t = a.lr / (1.f + a.decay * it);
    auto sgd = [&](float& p, float& v, float gi) {
      gi *= a.gscale;
      const float vn = a.momentum * v - lr_t * gi;
      v = vn;
      p += a.nesterov ? (a.momentum * vn - lr_t * gi) : vn;
    };
    if (tid < NWD && dj < O && f0 + dfl < a.filters) {
      sgd(wd[dj][dfl][dt4], vd[dj][dfl][dt4], gwd.x);
      sgd(wd[dj][dfl][dt4 + 1], vd[dj][dfl][dt4 + 1], gwd.y);
      sgd(wd[dj][dfl][dt4 + 2], vd[dj][dfl][dt4 + 2], gwd.z);
      sgd(wd[dj][dfl][dt4 + 3], vd[dj][dfl][dt4 + 3], gwd.w);
    }
    if (tid < CS_FPW * CS_KC) {
      const int fl = tid / CS_KC, kk = tid % CS_KC;
      if (kk <= taps && f0 + fl < a.filters) {
        float gs = 0.f;
        for (int t = 0; t < CS_T; ++t) gs += gwc[fl][kk][t];
        sgd(wc[fl][kk], vc[fl][kk], gs);
      }
    }
    if (tid >= 64 && tid < 64 + O) {  // dbd = sum over windows: 4 partial sums (w mod 4), fixed order
      // (one chain of B dependent LDS loads was ~0.6 us of this phase)
      const int j = tid - 64;
      float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int w = 0; w < B; w += 4) {  // B % 4 == 0 (launcher)
#pragma unroll
        for (int e = 0; e < 4; ++e) s4[e] += dout[w + e][j];
      }
      sgd(bd[j], vb[j], (s4[0] + s4[1]) + (s4[2] + s4[3]));
    }
    __syncthreads();
    stamp(8);
  }

  // ---- write back the owned parameters / velocities (worker 0: the dense bias too)
  for (int i = tid; i < CS_FPW * CS_KC; i += CS_NT) {
    const int fl = i / CS_KC, kk = i % CS_KC;
    const long e = (long)(f0 + fl) * CS_KC + kk;
    a.p[e] = wc[fl][kk];
    a.vel[e] = vc[fl][kk];
  }
  for (int i = tid; i < CS_OP * CS_T * CS_FPW; i += CS_NT) {
    const int j = i / (CS_T * CS_FPW), fl = (i / CS_T) % CS_FPW, t = i % CS_T;
    const long e = oWd + (long)j * CS_T * CS_FP + t * CS_FP + f0 + fl;
    a.p[e] = wd[j][fl][t];
    a.vel[e] = vd[j][fl][t];
  }
  if (wk == 0 && tid < CS_OP) {
    a.p[obd + tid] = bd[tid];
    a.vel[obd + tid] = vb[tid];
  }
  if (tid == 0) {
    if (wk == 0) {
      a.step[0] = it0 + (float)K;
      a.rng[0] = (long long)rng0 + K;
    }
    if (__hip_atomic_fetch_add((cs_g32*)(a.sync + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)G - 1) {
      __hip_atomic_store((cs_g32*)(a.sync + 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add((cs_g32*)(a.sync + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

bool launch_cnn_small(const CnnSmallArgs& a, hipStream_t s) {
  if (a.B < 4 || a.B > CS_MAXB || a.B % 4 != 0 || a.K <= 0 || a.K > 4095 || a.O < 1 || a.O > CS_OP || a.taps != CS_L - CS_T + 1 ||
      a.filters < 1 || a.filters > CS_FP)
    return false;
  const int G = (a.filters + CS_FPW - 1) / CS_FPW;
  if (G * CS_FPW > CS_FP || G > 28 || CS_P2 + 2 * CS_MAXB * CS_OP * 2 > kCnnSmallScratch) return false;
  if ((a.B * a.O + G - 1) / G > 48) return false;  // hop-1 outputs per worker (red2 rows)
  hipLaunchKernelGGL(cnn_small_kernel, dim3(G), dim3(CS_NT), 0, s, a);
  return true;
}

}  // namespace wf
