// wellflow — fused, weight-stationary forward (and backward, below) of the static / dynamic MLP regressor
// (BASELINE.json:8-10: F -> 256 -> 256 -> 1, ReLU, linear head, MSE; SURVEY.md §2.4 K10, K15,
// K16).
//
// Why: per layer, the generic GEMM path (gemm.hip) streams the activations through HBM
// and re-reads the 256 x 256 weight tile in every one of its 1024 short-lived workgroups,
// then a separate head kernel re-reads the last hidden layer: ~84 us of a 0.3 ms training
// step at 65,536 rows for ~71 MB of compulsory traffic. Here ONE launch does
//   Z1 = X W1^T + b1, H1 = relu(Z1); Z2 = H1 W2^T + b2, H2 = relu(Z2);
//   pred = H2 w3 + b3; (MSE) dy = s (pred - y), loss += (pred - y)^2
// with every weight resident in registers for the whole launch:
//  * grid <= 256 workgroups of 256 threads (4 waves, one per SIMD), persistent over
//    64-row chunks; wave w owns hidden units [64w, 64w + 64) of both layers.
//  * transposed products: C = W (A operand: weights, lane = unit) x act^T (B operand:
//    activations, lane = row), so each lane's MFMA result holds 4 CONSECUTIVE units of one
//    row — packed to 8 bytes it lands in the LDS activation tile [row][unit] that the next
//    layer reads as 16-byte B fragments (conflict-free XOR swizzle).
//  * W1 slice 16 VGPRs, W2 slice 128 VGPRs per lane (loaded once); H1 / H2 leave the CU
//    once each, as whole 16-byte row segments (they are the backward pass's saved
//    activations); the head dot product is reduced across lanes (DPP) and waves (LDS).
#include "common.h"
#include "gemm_core.h"
#include "kernels.h"

namespace wf {

namespace {
constexpr int MF_ROWS = 64;  // rows per chunk
constexpr int MF_H = 256;    // hidden width (both layers)

// [64 rows][256 units] bf16 tile, 16-B chunk c (units 8c..8c+7) of row r at chunk c ^ (r & 15)
// (32 chunks per row, 512-B rows): the B-fragment reads (16 rows x one chunk) hit 16 distinct
// 16-B bank groups, as do the row-wise copy-out reads.
__device__ __forceinline__ int tile_off(int row, int unit) {
  const int c = unit >> 3;
  return row * (MF_H * 2) + ((c ^ (row & 15)) << 4) + ((unit & 7) << 1);
}
// [64 rows][64 features] bf16 input tile (8 chunks per row, 128-B rows: rows r and r + 2
// share banks, so the chunk is swizzled by (row >> 1) & 7 — 16-row fragment reads of one
// chunk hit 16 distinct bank groups)
constexpr int MF_XROW = 128;
__device__ __forceinline__ int xtile_off(int row, int chunk) { return row * MF_XROW + ((chunk ^ ((row >> 1) & 7)) << 4); }
}  // namespace

template <int KT1>  // layer-1 K steps of 32 features: 1 (Fp <= 32) or 2 (Fp <= 64)
__global__ __launch_bounds__(256, 1) void mlp2_fwd_kernel(
    const bf16_t* __restrict__ X, int Fp, const bf16_t* __restrict__ W1, const float* __restrict__ b1,
    const bf16_t* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ w3,
    const float* __restrict__ b3, const float* __restrict__ y, bf16_t* __restrict__ H1, bf16_t* __restrict__ H2,
    unsigned* __restrict__ M2, float* __restrict__ dw3, float* __restrict__ db3, float* __restrict__ pred,
    float* __restrict__ dy, float* __restrict__ loss_sum, float dy_scale, int B) {
  __shared__ __attribute__((aligned(16))) char xs[MF_ROWS * MF_XROW];
  __shared__ __attribute__((aligned(16))) char h1s[MF_ROWS * MF_H * 2];
  __shared__ __attribute__((aligned(16))) char h2s[MF_ROWS * MF_H * 2];
  __shared__ float red[4][MF_ROWS];
  __shared__ float dys[MF_ROWS];
  __shared__ float lred[4];
  // mask mode (M2 != nullptr, training): H2 leaves the CU only as its ReLU bitmask (32 B per
  // row instead of 512 B) and the head gradients dw3 = H2^T dy, db3 = sum dy are accumulated
  // here, from the H2 tile still in LDS, so the backward never needs the H2 values
  const bool mask_mode = M2 != nullptr;
  const int ec = threadIdx.x & 31, erq = threadIdx.x >> 5;  // dw3 ownership: units 8ec .. 8ec + 7
  float dw3a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float db3a = 0.f;

  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = threadIdx.x >> 6;
  const int u0 = wid * 64;  // first unit of this wave

  // ---- stationary weights (A operand: lane = unit l15 of M-tile m, k 8g..8g+7)
  bf16x8 w1f[KT1][4], w2f[4][8];
  float bias1[4][4], bias2[4][4], w3v[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int u = u0 + 16 * m + l15;
#pragma unroll
    for (int k1 = 0; k1 < KT1; ++k1) {
      const int f0 = 32 * k1 + 8 * g;
      if (f0 + 8 <= Fp)
        w1f[k1][m] = *reinterpret_cast<const bf16x8*>(W1 + (size_t)u * Fp + f0);
      else
        w1f[k1][m] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) w2f[m][kt] = *reinterpret_cast<const bf16x8*>(W2 + (size_t)u * MF_H + 32 * kt + 8 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // C rows of this lane: units 16m + 4g + r
      const int uc = u0 + 16 * m + 4 * g + r;
      bias1[m][r] = b1[uc];
      bias2[m][r] = b2[uc];
      w3v[m][r] = w3[uc];
    }
  }
  const float bias3 = b3[0];
  float lsum = 0.f;

  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int row0 = ch * MF_ROWS;
    // ---- X chunk -> LDS, zero-padded to 32 * KT1 features (thread: row t >> 2, chunk t & 3 (+4))
#pragma unroll
    for (int k1 = 0; k1 < KT1; ++k1) {
      const int r = threadIdx.x >> 2, c = (threadIdx.x & 3) + 4 * k1, gr = row0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (gr < B && 8 * c + 8 <= Fp) v = *reinterpret_cast<const uint4*>(X + (size_t)gr * Fp + 8 * c);
      *reinterpret_cast<uint4*>(xs + xtile_off(r, c)) = v;
    }
    __syncthreads();

    // ---- layer 1: Z1^T (64 units x 64 rows per wave) = W1 x X^T, K = 32 * KT1
    f32x4 acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k1 = 0; k1 < KT1; ++k1)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(xs + xtile_off(16 * n + l15, 4 * k1 + g));
#pragma unroll
        for (int m = 0; m < 4; ++m)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[k1][m], xb, acc[m][n], 0, 0, 0);
      }
    // epilogue 1: + b1, relu, 4 units -> 8 B into the H1 tile
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        unsigned pk[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float v0 = fmaxf(acc[m][n][2 * q] + bias1[m][2 * q], 0.f);
          const float v1 = fmaxf(acc[m][n][2 * q + 1] + bias1[m][2 * q + 1], 0.f);
          pk[q] = (unsigned)f2bf(v0) | ((unsigned)f2bf(v1) << 16);
        }
        *reinterpret_cast<uint2*>(h1s + tile_off(16 * n + l15, u0 + 16 * m + 4 * g)) = make_uint2(pk[0], pk[1]);
      }
    __syncthreads();

    // ---- H1 tile -> HBM (saved for the backward): 64 rows x 512 B, 16-B stores
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = threadIdx.x + 256 * k, r = idx >> 5, c = idx & 31, gr = row0 + r;
      if (gr < B)
        *reinterpret_cast<uint4*>(H1 + (size_t)gr * MF_H + 8 * c) =
            *reinterpret_cast<const uint4*>(h1s + tile_off(r, 8 * c));
    }

    // ---- layer 2: Z2^T = W2 x H1^T, K = 256 (8 k-tiles)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      bf16x8 hb[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) hb[n] = *reinterpret_cast<const bf16x8*>(h1s + tile_off(16 * n + l15, 32 * kt + 8 * g));
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[m][kt], hb[n], acc[m][n], 0, 0, 0);
    }
    // epilogue 2: + b2, relu -> H2 tile; head partial sums per row
    float hp[4] = {0.f, 0.f, 0.f, 0.f};  // rows 16n + l15, this lane's 16 units
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // round to bf16 first: the head consumes exactly the H2 the backward will see
          v[r] = bf2f(f2bf(fmaxf(acc[m][n][r] + bias2[m][r], 0.f)));
          hp[n] += v[r] * w3v[m][r];
        }
        const unsigned p0 = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
        const unsigned p1 = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(h2s + tile_off(16 * n + l15, u0 + 16 * m + 4 * g)) = make_uint2(p0, p1);
      }
    // sum the 4 lane groups g (same row l15): lanes l15, l15 + 16, + 32, + 48
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      hp[n] += __shfl_xor(hp[n], 16, 64);
      hp[n] += __shfl_xor(hp[n], 32, 64);
    }
    if (g == 0) {
#pragma unroll
      for (int n = 0; n < 4; ++n) red[wid][16 * n + l15] = hp[n];
    }
    __syncthreads();

    // ---- H2 tile (or its ReLU bitmask) -> HBM; head + loss for the chunk's rows (threads 0..63)
    if (!mask_mode) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int idx = threadIdx.x + 256 * k, r = idx >> 5, c = idx & 31, gr = row0 + r;
        if (gr < B)
          *reinterpret_cast<uint4*>(H2 + (size_t)gr * MF_H + 8 * c) =
              *reinterpret_cast<const uint4*>(h2s + tile_off(r, 8 * c));
      }
    } else {
      // thread -> row t >> 2, units 64q .. 64q + 63 (q = t & 3) = mask words 2q, 2q + 1
      const int r = threadIdx.x >> 2, q = threadIdx.x & 3, gr = row0 + r;
      unsigned mw[2] = {0u, 0u};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint4 v = *reinterpret_cast<const uint4*>(h2s + tile_off(r, 64 * q + 8 * k));
        const unsigned w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int bit = 8 * k + e;
          if (bf2f((bf16_t)(w4[e >> 1] >> (16 * (e & 1)))) > 0.f) mw[bit >> 5] |= 1u << (bit & 31);
        }
      }
      if (gr < B) *reinterpret_cast<uint2*>(M2 + (size_t)gr * 8 + 2 * q) = make_uint2(mw[0], mw[1]);
    }
    if (threadIdx.x < MF_ROWS) {
      const int gr = row0 + threadIdx.x;
      if (gr < B) {
        const float p = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x] + bias3;
        pred[gr] = p;
        if (y != nullptr) {
          const float diff = p - y[gr];
          lsum += diff * diff;
          if (dy != nullptr) dy[gr] = dy_scale * diff;
          if (mask_mode) {
            dys[threadIdx.x] = dy_scale * diff;
            db3a += dy_scale * diff;
          }
        }
      } else if (mask_mode) {
        dys[threadIdx.x] = 0.f;
      }
    }
    if (mask_mode) {  // dw3 partials: H2 tile rows x dy
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = erq + 8 * q;
        const float gy = dys[r];
        const uint4 v = *reinterpret_cast<const uint4*>(h2s + tile_off(r, 8 * ec));
        const unsigned w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) dw3a[e] += gy * bf2f((bf16_t)(w4[e >> 1] >> (16 * (e & 1))));
      }
    }
    __syncthreads();  // xs / h1s / h2s / red / dys are rewritten by the next chunk
  }
  if (loss_sum != nullptr) {
    const float t = block_sum<256>(lsum, lred);
    if (threadIdx.x == 0 && t != 0.f) atomicAdd(loss_sum, t);
  }
  if (mask_mode) {
    // the 8 threads of one unit chunk (erq = 0..7) -> LDS [8][256], then one atomic per unit
    float* sd = reinterpret_cast<float*>(h1s);
#pragma unroll
    for (int e = 0; e < 8; ++e) sd[erq * MF_H + 8 * ec + e] = dw3a[e];
    __syncthreads();
    float s3 = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s3 += sd[q * MF_H + threadIdx.x];
    if (s3 != 0.f) atomicAdd(dw3 + threadIdx.x, s3);
    const float t3 = block_sum<256>(db3a, lred);
    if (threadIdx.x == 0 && t3 != 0.f) atomicAdd(db3, t3);
  }
}

// ----------------------------------------------------------------------------------------
// Fused backward of the same MLP, everything except the two weight-gradient GEMMs (which
// reduce over the whole batch and stay split-K GEMMs in gemm.hip):
//   dw3 += H2^T dy, db3 += sum dy                           (head)
//   dZ2 = (dy w3^T) * [H2 > 0]  -> HBM (bf16, dW2's operand), db2 += colsum dZ2
//   dZ1 = (dZ2 W2)  * [H1 > 0]  -> HBM (bf16, dW1's operand), db1 += colsum dZ1
// Replaces head_bwd_w + head_bwd_x + the dX GEMM (3 launches, dZ2 written then re-read, the
// 256 x 256 W2 tile re-read by each of ~4000 short workgroups): here H1 / H2 / dy are read
// once, dZ1 / dZ2 written once, and W2^T stays in registers.
//  * grid <= 256 workgroups of 4 waves, persistent over 64-row chunks. Wave w owns input
//    units k in [64w, 64w + 64) of dH1: A operand = W2^T rows (lane = k, K = u, gathered
//    once: 128 VGPRs), B operand = the dZ2 tile rows from LDS, exactly the forward's
//    transposed-product pattern, so each lane's result is 4 consecutive k of one row.
//  * elementwise phase: thread t always handles the 8-unit chunk c = t & 31 (rows
//    (t >> 5) + 8q), so its db2 / dw3 partials stay in registers across all chunks.
//  * the H1 tile is staged in LDS for the ReLU mask and overwritten in place by dZ1 (each
//    lane reads and writes the same 8 bytes), then copied out as 16-B row segments.
//  * dW1 = dZ1^T X (K = the batch) is accumulated here too when dW1 != nullptr: the dZ1 tile
//    [row][unit] and the X tile [row][feature] are both "MN-contiguous" images of operands
//    whose reduction index is the row, so their MFMA fragments come out of LDS with
//    ds_read_b64_tr_b16 (gemm_core.h) at per-lane addresses that follow this file's
//    swizzles; the 64 x Fp slice of dW1 per wave stays in registers across all chunks
//    (2 x 4 x NFT MFMAs per chunk), and dZ1 is then not written to HBM at all.
template <int NFT>  // 16-feature tiles of dW1 (1: Fp <= 16, 2: Fp <= 32): dW1 registers = 16 x NFT
__global__ __launch_bounds__(256, 1) void mlp2_bwd_kernel(
    const bf16_t* __restrict__ H1, const bf16_t* __restrict__ H2, const unsigned* __restrict__ M2,
    const float* __restrict__ dy,
    const float* __restrict__ w3, const bf16_t* __restrict__ W2, const bf16_t* __restrict__ X, int Fp,
    bf16_t* __restrict__ dZ1, bf16_t* __restrict__ dZ2, float* __restrict__ dW1, float* __restrict__ db1,
    float* __restrict__ db2, float* __restrict__ dw3, float* __restrict__ db3, int B) {
  __shared__ __attribute__((aligned(16))) char zs[MF_ROWS * MF_H * 2];  // dZ2 tile
  __shared__ __attribute__((aligned(16))) char hs[MF_ROWS * MF_H * 2];  // H1 tile -> dZ1 in place
  __shared__ __attribute__((aligned(16))) char xs[MF_ROWS * MF_XROW];   // X tile (dW1)
  __shared__ float lred[4];

  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = threadIdx.x >> 6;
  const int u0 = wid * 64;

  // ---- stationary W2^T (A operand: lane = input unit k = u0 + 16m + l15, K = output unit u)
  bf16x8 wt[4][8];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int k = u0 + 16 * m + l15;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int j = 0; j < 8; ++j) wt[m][kt][j] = (short)W2[(size_t)(32 * kt + 8 * g + j) * MF_H + k];
  }
  // ---- elementwise-phase ownership: units 8c .. 8c + 7
  const int c = threadIdx.x & 31, rq = threadIdx.x >> 5;
  float w3c[8], db2a[8], dw3a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    w3c[e] = w3[8 * c + e];
    db2a[e] = 0.f;
    dw3a[e] = 0.f;
  }
  float db3a = 0.f;
  float db1a[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) db1a[m][i] = 0.f;
  const bool fuse_dw1 = dW1 != nullptr;
  f32x4 dw1a[4][NFT];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int f = 0; f < NFT; ++f) dw1a[m][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per-lane tr-read coordinates (gemm_core.h MN fragment): tile row 8g + 4h + q (+ 32 kk),
  // 4 consecutive columns from 4p
  const int tq = (lane & 15) >> 2, tp = lane & 3;

  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int row0 = ch * MF_ROWS;
    // ---- dZ2 (+ head / db2 partials) from H2 and dy; H1 -> LDS (2 rows in flight per
    // thread: a full unroll keeps 8 x 2 row loads live and spills next to the 128-VGPR W2^T)
#pragma unroll 2
    for (int q = 0; q < 8; ++q) {
      const int r = rq + 8 * q, gr = row0 + r;
      uint4 h2v = make_uint4(0, 0, 0, 0), h1v = make_uint4(0, 0, 0, 0);
      unsigned mb = 0u;  // mask mode: ReLU bits of units 8c .. 8c + 7
      float gy = 0.f;
      if (gr < B) {
        if (M2 == nullptr)
          h2v = *reinterpret_cast<const uint4*>(H2 + (size_t)gr * MF_H + 8 * c);
        else
          mb = M2[(size_t)gr * 8 + (c >> 2)] >> (8 * (c & 3));
        h1v = *reinterpret_cast<const uint4*>(H1 + (size_t)gr * MF_H + 8 * c);
        gy = dy[gr];
      }
      if (c == 0 && M2 == nullptr) db3a += gy;  // mask mode: the forward did the head gradients
      const unsigned hw[4] = {h2v.x, h2v.y, h2v.z, h2v.w};
      unsigned zw[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        unsigned pk = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = 2 * p + h;
          bool on;
          if (M2 == nullptr) {
            const float hv = bf2f((bf16_t)(hw[p] >> (16 * h)));
            dw3a[e] += gy * hv;
            on = hv > 0.f;
          } else {
            on = (mb >> e) & 1u;
          }
          const bf16_t zb = f2bf(on ? gy * w3c[e] : 0.f);
          db2a[e] += bf2f(zb);
          pk |= (unsigned)zb << (16 * h);
        }
        zw[p] = pk;
      }
      const uint4 zv = make_uint4(zw[0], zw[1], zw[2], zw[3]);
      *reinterpret_cast<uint4*>(zs + tile_off(r, 8 * c)) = zv;
      *reinterpret_cast<uint4*>(hs + tile_off(r, 8 * c)) = h1v;
      if (gr < B) *reinterpret_cast<uint4*>(dZ2 + (size_t)gr * MF_H + 8 * c) = zv;
    }
    if (fuse_dw1) {  // X chunk -> LDS, zero-padded to 32 features (as in the forward)
      const int r = threadIdx.x >> 2, xc = threadIdx.x & 3, gr = row0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (gr < B && 8 * xc + 8 <= Fp) v = *reinterpret_cast<const uint4*>(X + (size_t)gr * Fp + 8 * xc);
      *reinterpret_cast<uint4*>(xs + xtile_off(r, xc)) = v;
    }
    __syncthreads();

    // ---- dH1^T (64 k x 64 rows per wave) = W2^T x dZ2^T, K = 256
    f32x4 acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      bf16x8 zb[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) zb[n] = *reinterpret_cast<const bf16x8*>(zs + tile_off(16 * n + l15, 32 * kt + 8 * g));
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wt[m][kt], zb[n], acc[m][n], 0, 0, 0);
    }
    // ---- ReLU mask from the H1 tile, dZ1 back into the same 8 bytes, db1 partials
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int r = 16 * n + l15;
        uint2* p = reinterpret_cast<uint2*>(hs + tile_off(r, u0 + 16 * m + 4 * g));
        const uint2 hv = *p;
        const unsigned hw2[2] = {hv.x, hv.y};
        unsigned ow[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          unsigned pk = 0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int i = 2 * q + h;
            const bool on = bf2f((bf16_t)(hw2[q] >> (16 * h))) > 0.f && row0 + r < B;
            const bf16_t vb = f2bf(on ? acc[m][n][i] : 0.f);
            db1a[m][i] += bf2f(vb);
            pk |= (unsigned)vb << (16 * h);
          }
          ow[q] = pk;
        }
        *p = make_uint2(ow[0], ow[1]);
      }
    __syncthreads();
    if (fuse_dw1) {
      // ---- dW1^T slice (64 units x Fp per wave) += dZ1^T X over this chunk's 64 rows
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[4], bfr[NFT];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = 32 * kk + 8 * g + 4 * h + tq;
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_bf16x4*)(hs + tile_off(r, u0 + 16 * m + 4 * tp)));
#pragma unroll
            for (int e = 0; e < 4; ++e) af[m][4 * h + e] = v[e];
          }
#pragma unroll
          for (int f = 0; f < NFT; ++f) {
            const int f0 = 16 * f + 4 * tp;
            const bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_bf16x4*)(xs + xtile_off(r, f0 >> 3) + ((f0 & 7) << 1)));
#pragma unroll
            for (int e = 0; e < 4; ++e) bfr[f][4 * h + e] = v[e];
          }
        }
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int f = 0; f < NFT; ++f)
            dw1a[m][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[f], dw1a[m][f], 0, 0, 0);
      }
      __syncthreads();  // zs / hs / xs are rewritten by the next chunk
      continue;        // dZ1 itself is not needed outside this kernel
    }
    // ---- dZ1 tile -> HBM
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = threadIdx.x + 256 * k, r = idx >> 5, cc = idx & 31, gr = row0 + r;
      if (gr < B)
        *reinterpret_cast<uint4*>(dZ1 + (size_t)gr * MF_H + 8 * cc) =
            *reinterpret_cast<const uint4*>(hs + tile_off(r, 8 * cc));
    }
    __syncthreads();  // zs / hs are rewritten by the next chunk
  }

  // ---- reductions. db1: lanes of one g share k = u0 + 16m + 4g + i -> sum over l15
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = db1a[m][i];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if (l15 == 0 && v != 0.f) atomicAdd(db1 + u0 + 16 * m + 4 * g + i, v);
    }
  // dW1 (C layout: lane holds units u0 + 16m + 4g + i, feature l15 + 16f)
  if (fuse_dw1) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int f = 0; f < NFT; ++f) {
        const int ft = l15 + 16 * f;
        if (ft < Fp)
#pragma unroll
          for (int i = 0; i < 4; ++i) atomicAdd(dW1 + (size_t)(u0 + 16 * m + 4 * g + i) * Fp + ft, dw1a[m][f][i]);
      }
  }
  // db2 / dw3: the 8 threads of one chunk c (rq = 0..7) -> LDS [8][256] x 2, then one per unit
  float* sd = reinterpret_cast<float*>(zs);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sd[rq * MF_H + 8 * c + e] = db2a[e];
    sd[8 * MF_H + rq * MF_H + 8 * c + e] = dw3a[e];
  }
  __syncthreads();
  {
    const int u = threadIdx.x;
    float s2 = 0.f, s3 = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      s2 += sd[q * MF_H + u];
      s3 += sd[8 * MF_H + q * MF_H + u];
    }
    if (s2 != 0.f) atomicAdd(db2 + u, s2);
    if (s3 != 0.f) atomicAdd(dw3 + u, s3);
  }
  const float t3 = block_sum<256>(db3a, lred);
  if (threadIdx.x == 0 && t3 != 0.f) atomicAdd(db3, t3);
}

bool launch_mlp2_bwd(const bf16_t* H1, const bf16_t* H2, const unsigned* M2, const float* dy, const float* w3, const bf16_t* W2,
                     const bf16_t* X, int Fp, bf16_t* dZ1, bf16_t* dZ2, float* dW1, float* db1, float* db2,
                     float* dw3, float* db3, int B, hipStream_t s) {
  if (B <= 0 || (dW1 != nullptr && (X == nullptr || Fp > 32 || Fp % 8 != 0))) return false;
  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int grid = nchunks < cus ? nchunks : cus;
  if (Fp <= 16)
    hipLaunchKernelGGL(mlp2_bwd_kernel<1>, dim3(grid), dim3(256), 0, s, H1, H2, M2, dy, w3, W2, X, Fp, dZ1, dZ2, dW1,
                       db1, db2, dw3, db3, B);
  else
    hipLaunchKernelGGL(mlp2_bwd_kernel<2>, dim3(grid), dim3(256), 0, s, H1, H2, M2, dy, w3, W2, X, Fp, dZ1, dZ2, dW1,
                       db1, db2, dw3, db3, B);
  return true;
}

bool launch_mlp2_fwd(const bf16_t* X, int Fp, const bf16_t* W1, const float* b1, const bf16_t* W2, const float* b2,
                     const float* w3, const float* b3, const float* y, bf16_t* H1, bf16_t* H2, unsigned* M2,
                     float* dw3, float* db3, float* pred, float* dy, float* loss_sum, float dy_scale, int B,
                     hipStream_t s) {
  if (Fp > 64 || Fp % 8 != 0 || B <= 0) return false;
  if (M2 != nullptr && (y == nullptr || dw3 == nullptr || db3 == nullptr)) return false;
  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int grid = nchunks < cus ? nchunks : cus;
  if (Fp <= 32)
    hipLaunchKernelGGL(mlp2_fwd_kernel<1>, dim3(grid), dim3(256), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y, H1, H2,
                       M2, dw3, db3, pred, dy, loss_sum, dy_scale, B);
  else
    hipLaunchKernelGGL(mlp2_fwd_kernel<2>, dim3(grid), dim3(256), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y, H1, H2,
                       M2, dw3, db3, pred, dy, loss_sum, dy_scale, B);
  return true;
}

}  // namespace wf
