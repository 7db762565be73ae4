// wellflow — LSTM kernels (BASELINE.json config 5:
// seq-len 64, hidden 512, seq-to-one regression, bf16 on MFMA).
//
// Design (MI355X-first, not a cuDNN translation):
//  * The input projection is not hoisted into a [T,B,4H] tensor (2 GB at B=8192):
//    every step multiplies the concatenated row [x_t | 1 | 0.. | h_{t-1}] (KA = KX + H
//    columns, KX = 64) by one weight matrix Wp [4H][KA] whose "1" column carries the
//    bias. The whole cell is one GEMM + fused epilogue per timestep; the weight gradient
//    for W_ih, W_hh and the bias becomes ONE big GEMM over all (t, b) at the end.
//  * Gate columns are permuted so that a wave's 64-column N tile holds gates i,f,g,o of
//    the same 16 hidden units: with the 16x16 MFMA C map each lane then owns all four
//    gate pre-activations of its (row, unit) pairs and the cell update needs no LDS
//    exchange.  column p <-> (gate, unit):  unit = (p>>6)*16 + (p&15),  gate = (p>>4)&3.
//  * XH[t] (bf16 [B][KA]) is both the GEMM A operand of step t and the saved input of
//    the weight-gradient GEMM; step t writes h_t straight into XH[t+1][:, KX:].
//  * Backward step t is the GEMM dh_t = dG_{t+1} * W_hh (B operand WhhT = W_hh^T kept as
//    a bf16 shadow, K-contiguous) whose epilogue runs the cell backward for step t and
//    writes dG_t, so the time recurrence costs T-1 GEMM launches and no extra passes.
#include "gemm_core.h"
#include "kernels.h"
#include "lstm_layout.h"

namespace wf {

// XH[t][b][0:KX] = [x[b][t][0:F], 1, 0, ...]. One lane per 16-B chunk of a destination
// row (KX/8 lanes per row, rows of one timestep consecutive): every store instruction
// writes whole 128-B lines of 8 rows instead of 64 partial lines (the thread-per-row
// version ran at 1.6 TB/s).
// cpr = 16-B chunks written per row: all KX/8 (full: the constant 1 column and the zero
// padding too) or only the ones holding features and the 1 column (the rest of the x block is
// constant, so after one full pack of a buffer the per-step pack writes 3 of 8 chunks at F = 16)
// win != nullptr: x is a per-row feature table [nrows][F] and batch row b is the length-T
// window starting at row starts[idx[b]] (data/features.py SeriesWindows read in place: the job's
// per-step torch gather of the [B][T][F] windows cost ~150 us of a 4.2-ms step)
struct PackWin {
  const long* starts;
  const long* idx;
  long nwin, nrows;
};

__global__ void lstm_pack_x_kernel(const float* __restrict__ x, bf16_t* __restrict__ XH,
                                   LstmDims d, int cpr, PackWin win) {
  const int KA = d.KX + d.H, CPR = cpr;
  const long total = (long)d.T * d.B * CPR;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int c = (int)(idx % CPR) * 8;
    const long row = idx / CPR;  // = t * B + b
    const long b = row % d.B;
    const int t = (int)(row / d.B);
    const float* src;
    if (win.idx != nullptr) {  // ids clamped into the tables (a bad id reads a valid row, never faults)
      long w = win.idx[b];
      w = w < 0 ? 0 : (w >= win.nwin ? win.nwin - 1 : w);
      long r0 = win.starts[w];
      r0 = r0 < 0 ? 0 : (r0 > win.nrows - d.T ? win.nrows - d.T : r0);
      src = x + (r0 + t) * d.F;
    } else {
      src = x + (b * d.T + t) * d.F;
    }
    unsigned pk[4];
    // 8 features: two 16-B loads (rows are 16-B aligned when F % 4 == 0 and x is)
    if ((d.F & 3) == 0 && c + 8 <= d.F && ((uintptr_t)x & 15u) == 0) {
      const float4 lo = *reinterpret_cast<const float4*>(src + c);
      const float4 hi = *reinterpret_cast<const float4*>(src + c + 4);
      pk[0] = (unsigned)f2bf(lo.x) | ((unsigned)f2bf(lo.y) << 16);
      pk[1] = (unsigned)f2bf(lo.z) | ((unsigned)f2bf(lo.w) << 16);
      pk[2] = (unsigned)f2bf(hi.x) | ((unsigned)f2bf(hi.y) << 16);
      pk[3] = (unsigned)f2bf(hi.z) | ((unsigned)f2bf(hi.w) << 16);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k0 = c + 2 * e, k1 = k0 + 1;
        const float v0 = k0 < d.F ? src[k0] : (k0 == d.F ? 1.f : 0.f);
        const float v1 = k1 < d.F ? src[k1] : (k1 == d.F ? 1.f : 0.f);
        pk[e] = (unsigned)f2bf(v0) | ((unsigned)f2bf(v1) << 16);
      }
    }
    *reinterpret_cast<uint4*>(XH + row * KA + c) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  }
}

void launch_lstm_pack_x(const float* x, bf16_t* XH, LstmDims d, hipStream_t s, bool full, const long* starts,
                        const long* idx, long nwin, long nrows) {
  // per-step packs round the chunks written up to whole 64-B segments (4 chunks; the rest of the
  // block is the constant zero padding): 48 of a row's 128-B x block left a partial 32-B sector
  int cpr = full ? (d.KX >> 3) : ((d.F + 1 + 7) / 8 + 3) / 4 * 4;
  if (cpr > (d.KX >> 3)) cpr = d.KX >> 3;
  const long total = (long)d.T * d.B * cpr;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(lstm_pack_x_kernel, dim3(blocks), dim3(256), 0, s, x, XH, d, cpr, PackWin{starts, idx, nwin, nrows});
}

// STAGES == 0: register-staged mainloop (any batch); STAGES >= 2: direct-to-LDS ring
// (requires B % BM == 0, checked by the launcher).
template <int BM, int WM, int WN, int STAGES>
__global__ __launch_bounds__(64 * WM * WN) void lstm_fwd_step_kernel(int t, bf16_t* __restrict__ XH,
                                                            const bf16_t* __restrict__ Wp,
                                                            bf16_t* __restrict__ Cst,
                                                            bf16_t* __restrict__ S, float* __restrict__ cf32,
                                                            LstmDims d) {
  // wave N tile must be 64 = 4 gates x 16 units
  using C = GemmCfg<BM, 64 * WN, K_CONTIG, K_CONTIG, WM, WN>;
  constexpr int LDSB = STAGES * C::STAGE > C::LDS_BYTES ? STAGES * C::STAGE : C::LDS_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  const int KA = d.KX + d.H, G = 4 * d.H;
  const int tiles_n = G / C::BN;
  const int L = d.xcd_map ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int m0 = (L / tiles_n) * C::BM, n0 = (L % tiles_n) * C::BN;
  const bf16_t* A = XH + (size_t)t * d.B * KA;

  const AccCoord<C> cc(m0, n0);
  const int lane = threadIdx.x & 63;
  const int u = (cc.nb >> 6) * 16 + (lane & 15);
  const int Bp = fn_rows(d.B);
  // c_{t-1} in fp32 from the in-place state slab cf32 (FN layout; every element is read and
  // rewritten by the same lane, c_{-1} = 0); the bf16 history Cst is for the backward only

  f32x4 acc[C::TM][C::TN];
  if constexpr (STAGES >= 2)
    gemm_mainloop_glds2<C, STAGES>(A, KA, Wp, KA, 0, KA / 64, m0, n0, smem, acc);
  else
    gemm_mainloop<C>(A, KA, d.B, Wp, KA, G, 0, KA, m0, n0, smem, acc);

  bf16_t* cnext = Cst + (size_t)(t + 1) * Bp * d.H;
  bf16_t* hnext = XH + (size_t)(t + 1) * d.B * KA + d.KX;
  bf16_t* St = S + (size_t)t * Bp * G;
#pragma unroll
  for (int i = 0; i < C::TM; ++i) {
    const int mrow0 = cc.mb + i * 16;
    if (mrow0 >= d.B) continue;
    const size_t blk = fn_block(mrow0, u, d.H);
    float4* cst = reinterpret_cast<float4*>(cf32 + blk * 256 + lane * 4);
    const float4 cp = t > 0 ? *cst : make_float4(0.f, 0.f, 0.f, 0.f);
    const float cpv[4] = {cp.x, cp.y, cp.z, cp.w};
    float cv[4];
    unsigned pk[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ig = sigmoid_pre(acc[i][0][r]);  // Wp carries the gate scales (pack kernel)
      const float fg = sigmoid_pre(acc[i][1][r]);
      const float gg = tanh_pre(acc[i][2][r]);
      const float og = sigmoid_pre(acc[i][3][r]);
      const float c = fg * cpv[r] + ig * gg;
      cv[r] = c;
      pk[2 * r] = (unsigned)f2bf(ig) | ((unsigned)f2bf(fg) << 16);
      pk[2 * r + 1] = (unsigned)f2bf(gg) | ((unsigned)f2bf(og) << 16);
      const int m = mrow0 + 4 * (lane >> 4) + r;
      if (m < d.B) hnext[(size_t)m * KA + u] = f2bf(og * tanhf_(c));
    }
    *cst = make_float4(cv[0], cv[1], cv[2], cv[3]);
    *reinterpret_cast<uint2*>(cnext + blk * 256 + lane * 4) = make_uint2(pk_bf16(cv[0], cv[1]), pk_bf16(cv[2], cv[3]));
    bf16_t* sb = St + blk * 1024 + lane * 8;  // FN S halves (lstm_layout.h kFnSHalf)
    st16(sb, make_uint4(pk[0], pk[1], pk[2], pk[3]), d.nt);
    st16(sb + kFnSHalf, make_uint4(pk[4], pk[5], pk[6], pk[7]), d.nt);
  }
}

template <int BM, int WM, int WN, int STAGES = 0>
static void fwd_cfg(int t, bf16_t* XH, const bf16_t* Wp, bf16_t* Cst, bf16_t* S, float* cf32, LstmDims d,
                    hipStream_t s) {
  if (STAGES >= 2 && (d.B % BM != 0 || (4 * d.H) % (64 * WN) != 0)) {  // partial tiles
    fwd_cfg<BM, WM, WN, 0>(t, XH, Wp, Cst, S, cf32, d, s);
    return;
  }
  const int tiles = ((d.B + BM - 1) / BM) * (4 * d.H / (64 * WN));
  hipLaunchKernelGGL((lstm_fwd_step_kernel<BM, WM, WN, STAGES>), dim3(tiles), dim3(64 * WM * WN), 0,
                     s, t, XH, Wp, Cst, S, cf32, d);
}

// Per-step forward (the fallback of shapes the persistent forward does not take). Two tile
// shapes stay built: 6 = 256x256, 8 waves, 2-stage glds ring (tools/tune_lstm.py, the engine
// default) and 0 = 128x128 register-staged (any batch); the round-1 tuning zoo is retired.
void launch_lstm_fwd_step(int t, bf16_t* XH, const bf16_t* Wp, bf16_t* Cst, bf16_t* S, float* cf32,
                          LstmDims d, hipStream_t s) {
  if (d.fwd_variant == 6)
    fwd_cfg<256, 2, 4, 2>(t, XH, Wp, Cst, S, cf32, d, s);
  else
    fwd_cfg<128, 2, 2>(t, XH, Wp, Cst, S, cf32, d, s);
}

// Cell backward for the 4 rows (mrow0 + 4*(lane>>4) + r) x unit u of step t held by this
// lane, given dh for them: reads the lane's fragment-native S / C / dc-carry slots with
// 16-B vector accesses, updates the carry and writes the gate gradients into DG[t]
// (row-major, dg_col order: it is the next GEMM's A operand and the dW GEMM's M side).
template <bool FIRST = false>  // FIRST: step T-1, the dc carry starts at zero (not read)
__device__ __forceinline__ void cell_bwd4(int t, int mrow0, int u, int lane, const float (&dh)[4],
                                          const bf16_t* __restrict__ Cst,
                                          const bf16_t* __restrict__ S, bf16_t* __restrict__ DG,
                                          float* __restrict__ dcarry, const LstmDims& d) {
  const int G = 4 * d.H, Bp = fn_rows(d.B);
  const size_t blk = fn_block(mrow0, u, d.H);
  const bf16_t* sb = S + (size_t)t * Bp * G + blk * 1024 + lane * 8;  // FN S halves (lstm_layout.h)
  const uint4 s0 = ld16(sb, d.nt), s1 = ld16(sb + kFnSHalf, d.nt);
  const unsigned pk[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  // only c_{t-1} is read: c_t = f * c_{t-1} + i * g is recomputed from the saved gates
  // (the same bf16 gates every other term of the cell backward uses), which drops one
  // 16.8 MB state read per step at B = 8192
  // (bf16 history: 4 values = 8 B per lane)
  const uint2 p2 = *reinterpret_cast<const uint2*>(Cst + (size_t)t * Bp * d.H + blk * 256 + lane * 4);
  const float4 p4 = make_float4(__uint_as_float(p2.x << 16), __uint_as_float(p2.x & 0xffff0000u),
                                __uint_as_float(p2.y << 16), __uint_as_float(p2.y & 0xffff0000u));
  float4* dcp = reinterpret_cast<float4*>(dcarry + blk * 256 + lane * 4);
  const float4 k4 = FIRST ? make_float4(0.f, 0.f, 0.f, 0.f) : *dcp;
  const float pv[4] = {p4.x, p4.y, p4.z, p4.w};
  const float kv[4] = {k4.x, k4.y, k4.z, k4.w};
  float nk[4];
  bf16_t* dgt = DG + (size_t)t * d.B * G;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float ig = bf2f((bf16_t)(pk[2 * r] & 0xffff)), fg = bf2f((bf16_t)(pk[2 * r] >> 16));
    const float gg = bf2f((bf16_t)(pk[2 * r + 1] & 0xffff)), og = bf2f((bf16_t)(pk[2 * r + 1] >> 16));
    const float tc = tanhf_(fg * pv[r] + ig * gg);
    const float dc = kv[r] + dh[r] * og * (1.f - tc * tc);
    nk[r] = dc * fg;
    const int m = mrow0 + 4 * (lane >> 4) + r;
    if (m < d.B) {
      uint2 v;
      v.x = (unsigned)f2bf(dc * gg * ig * (1.f - ig)) | ((unsigned)f2bf(dc * pv[r] * fg * (1.f - fg)) << 16);
      v.y = (unsigned)f2bf(dc * ig * (1.f - gg * gg)) | ((unsigned)f2bf(dh[r] * tc * og * (1.f - og)) << 16);
      *reinterpret_cast<uint2*>(dgt + (size_t)m * G + dg_col(0, u)) = v;
    }
  }
  *dcp = make_float4(nk[0], nk[1], nk[2], nk[3]);
}

// t = T-1: dh comes from the regression head, dh[m][u] = dy[m] * w_out[u]; the carry
// starts at 0. One thread per (fragment-native block, lane) = 4 rows of one unit.
__global__ void lstm_bwd_last_kernel(const bf16_t* __restrict__ Cst, const bf16_t* __restrict__ S,
                                     bf16_t* __restrict__ DG, float* __restrict__ dcarry,
                                     const float* __restrict__ dy, const float* __restrict__ w_out,
                                     LstmDims d) {
  const int ub = d.H >> 4;
  const long total = (long)(fn_rows(d.B) >> 4) * ub * 64;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int lane = idx & 63;
    const long blk = idx >> 6;
    const int mrow0 = (int)(blk / ub) * 16, u = (int)(blk % ub) * 16 + (lane & 15);
    float dh[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mrow0 + 4 * (lane >> 4) + r;
      dh[r] = m < d.B ? dy[m] * w_out[u] : 0.f;
    }
    cell_bwd4<true>(d.T - 1, mrow0, u, lane, dh, Cst, S, DG, dcarry, d);
  }
}

template <int BM, int BN, int WM, int WN, int STAGES>
__global__ __launch_bounds__(64 * WM * WN) void lstm_bwd_step_kernel(int t, const bf16_t* __restrict__ WhhT,
                                                            const bf16_t* __restrict__ Cst,
                                                            const bf16_t* __restrict__ S,
                                                            bf16_t* __restrict__ DG,
                                                            float* __restrict__ dcarry, LstmDims d) {
  using C = GemmCfg<BM, BN, K_CONTIG, K_CONTIG, WM, WN>;
  constexpr int LDSB = STAGES * C::STAGE > C::LDS_BYTES ? STAGES * C::STAGE : C::LDS_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  const int G = 4 * d.H;
  const int tiles_n = d.H / C::BN;
  const int L = d.xcd_map ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int m0 = (L / tiles_n) * C::BM, n0 = (L % tiles_n) * C::BN;
  const bf16_t* A = DG + (size_t)(t + 1) * d.B * G;

  f32x4 acc[C::TM][C::TN];
  if constexpr (STAGES >= 2)
    gemm_mainloop_glds2<C, STAGES>(A, G, WhhT, G, 0, G / 64, m0, n0, smem, acc);
  else
    gemm_mainloop<C>(A, G, d.B, WhhT, G, d.H, 0, G, m0, n0, smem, acc);

  const AccCoord<C> cc(m0, n0);
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    const int u = cc.col(j);
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
      const int mrow0 = cc.mb + i * 16;
      if (mrow0 >= d.B) continue;
      const float dh[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      cell_bwd4(t, mrow0, u, lane, dh, Cst, S, DG, dcarry, d);
    }
  }
}

template <int BM, int BN, int WM = 2, int WN = 2, int STAGES = 0>
static void bwd_cfg(int t, const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S, bf16_t* DG,
                    float* dcarry, LstmDims d, hipStream_t s) {
  if (STAGES >= 2 && d.B % BM != 0) {
    bwd_cfg<BM, BN, WM, WN, 0>(t, WhhT, Cst, S, DG, dcarry, d, s);
    return;
  }
  const int tiles = ((d.B + BM - 1) / BM) * (d.H / BN);
  hipLaunchKernelGGL((lstm_bwd_step_kernel<BM, BN, WM, WN, STAGES>), dim3(tiles), dim3(64 * WM * WN),
                     0, s, t, WhhT, Cst, S, DG, dcarry, d);
}

void launch_lstm_bwd_step(int t, const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S,
                          bf16_t* DG, float* dcarry, const float* dy, const float* w_out,
                          LstmDims d, hipStream_t s) {
  if (t == d.T - 1) {
    const long total = (long)(fn_rows(d.B) >> 4) * (d.H >> 4) * 64;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(lstm_bwd_last_kernel, dim3(blocks), dim3(256), 0, s, Cst, S, DG, dcarry,
                       dy, w_out, d);
    return;
  }
  // two tile shapes stay built (the tuning zoo of round 1 is retired): 8 = 128x128, 8 waves,
  // 3-stage glds ring (tools/tune_lstm.py, the engine default), 0 = 128x128 register-staged
  if (d.bwd_variant == 8)
    bwd_cfg<128, 128, 2, 4, 3>(t, WhhT, Cst, S, DG, dcarry, d, s);
  else
    bwd_cfg<128, 128>(t, WhhT, Cst, S, DG, dcarry, d, s);
}

// fp32 master W [G][KA] (rows in dg_col order) -> bf16 Wp [G][KA] (rows in gate_col order,
// the forward's, each gate row pre-scaled for sigmoid_pre / tanh_pre: common.h) and WhhT
// [H][G] (columns in dg_col order, the backward's, unscaled).
__global__ void lstm_pack_weights_kernel(const float* __restrict__ W, bf16_t* __restrict__ Wp,
                                         bf16_t* __restrict__ WhhT, LstmDims d) {
  const int KA = d.KX + d.H, G = 4 * d.H;
  const long total = (long)G * KA;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int k = idx % KA, p = idx / KA;
    const float w = W[idx];
    const float sc = (p & 3) == 2 ? kLstmTanhScale : kLstmSigScale;
    Wp[(size_t)gate_col(p & 3, p >> 2) * KA + k] = f2bf(w * sc);
    if (k >= d.KX) WhhT[(size_t)(k - d.KX) * G + p] = f2bf(w);
  }
}

void launch_lstm_pack_weights(const float* W, bf16_t* Wp, bf16_t* WhhT, LstmDims d, hipStream_t s) {
  const long total = (long)4 * d.H * (d.KX + d.H);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(lstm_pack_weights_kernel, dim3(blocks), dim3(256), 0, s, W, Wp, WhhT, d);
}

}  // namespace wf
