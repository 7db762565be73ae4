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
#include <cstdlib>

#include "common.h"
#include "gemm_core.h"
#include "kernels.h"
#include "mlp_tiles.h"

namespace wf {

namespace {
// WELLFLOW_MLP_PRIO bit mask: s_setprio(1) around the MFMA clusters of 1 forward, 2 backward,
// 4 dW2 (8-wave kernels)
int mlp_prio() {
  static const int p = diag_env_int("WELLFLOW_MLP_PRIO", 0);  // A/B, WF_DIAG builds only
  return p;
}
// WELLFLOW_MLP_DBG: timing-only switches of the 8-wave forward / backward (results are wrong).
// Diagnostic builds only (WF_DIAG, WELLFLOW_DIAG_BUILD=1): a production object ignores the
// variable, and kMlpDbgMask = 0 folds the branches out of the kernels (round-3 VERDICT weak #3).
#ifdef WF_DIAG
constexpr int kMlpDbgMask = ~0;
int mlp_dbg() {
  static const int d = [] {
    const char* e = std::getenv("WELLFLOW_MLP_DBG");
    return e == nullptr ? 0 : std::atoi(e);
  }();
  return d;
}
#else
constexpr int kMlpDbgMask = 0;
int mlp_dbg() { return 0; }
#endif
}  // namespace
constexpr int MF_ROWS_PUB = MF_ROWS;

// Spread reduction of the training kernels' batch sums (kernels.h kMlpRed*): every workgroup of
// the 8-wave forward / backward used to atomically add its partial loss, dw3, db3, db1, db2
// and dW1 straight into the gradient, i.e. 256 adders per address at the same moment, and the
// atomic unit serialises same-address adds: ~25 us of each ~36 us one-chunk-per-workgroup
// launch (WELLFLOW_MLP_DBG=1 A/B, profiles/r3_summary.md). They now add into copy
// blockIdx % kMlpRedCopies (64) of a scratch row (4 adders per address); dW2's 64 split-K adders
// per address go to copy split % 4; the backward's dW1 (4096 values per workgroup, too many
// atomic wave-instructions per CU) goes out as plain per-workgroup rows. mlp2_reduce_kernel
// sums copies and rows into the gradients and re-zeroes the copies.
__global__ __launch_bounds__(256) void mlp2_reduce_kernel(float* __restrict__ red, int Fp, int nwg, int slab_blocks,
                                                          float* __restrict__ loss_sum,
                                                          float* __restrict__ db3, float* __restrict__ dw3,
                                                          float* __restrict__ db1, float* __restrict__ db2,
                                                          float* __restrict__ dW1, float* __restrict__ dW2, int dw2_rows) {
  if ((int)blockIdx.x < slab_blocks) {
    // dW1 slab: block b sums 16 consecutive entries over the nwg (<= 256) workgroup rows in 16
    // row groups, every thread's 16 loads independent (one latency round, not a chain)
    __shared__ float part[16][16];
    const int o = blockIdx.x * 16 + (threadIdx.x & 15), rg = threadIdx.x >> 4;
    const float* sl = red + kMlpRedSlabOff;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (o < 256 * Fp) {
#pragma unroll
      for (int k = 0; k < kMlpRedSlabRows / 16; ++k) {
        const int r = rg + 16 * k;
        if (r < nwg) v[k & 3] += sl[(size_t)r * kMlpRedSlabRow + o];
      }
    }
    part[rg][threadIdx.x & 15] = (v[0] + v[1]) + (v[2] + v[3]);
    __syncthreads();
    if (rg == 0 && o < 256 * Fp) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) t += part[q][threadIdx.x];
      if (dW1 != nullptr && t != 0.f) dW1[o] += t;
    }
    return;
  }
  const int na = kMlpRedDW1;         // the small sums (no dW1 in the copies)
  const int nA = (na + 255) / 256;  // blocks of the small sums
  const int bx = (int)blockIdx.x - slab_blocks;
  if (bx < nA) {
    const int i = bx * 256 + threadIdx.x;
    if (i >= na) return;
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kMlpRedCopies; ++c) {
      v += red[c * kMlpRedRow + i];
      red[c * kMlpRedRow + i] = 0.f;
    }
    float* dst = i == kMlpRedLoss ? loss_sum
                 : i == kMlpRedDb3 ? db3
                 : i < kMlpRedDb1  ? (dw3 != nullptr ? dw3 + (i - kMlpRedDw3) : nullptr)
                 : i < kMlpRedDb2  ? (db1 != nullptr ? db1 + (i - kMlpRedDb1) : nullptr)
                                   : (db2 != nullptr ? db2 + (i - kMlpRedDb2) : nullptr);
    if (dst != nullptr && v != 0.f) *dst += v;
    return;
  }
  // dW2: block = 64 consecutive entries x 4 row groups: group 0 also sums (and re-zeroes) the
  // kMlpRedCopies2 atomic copies; every group sums every 4th of the dW2 kernel's slab rows
  // (plain stores, overwritten every step: not zeroed); the groups meet in LDS
  __shared__ float part2[4][64];
  const int e = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int j = (bx - nA) * 64 + e;
  float v = 0.f;
  if (q == 0) {
    float* r2 = red + kMlpRedCopies * kMlpRedRow;
#pragma unroll
    for (int c = 0; c < kMlpRedCopies2; ++c) {
      v += r2[c * 65536 + j];
      r2[c * 65536 + j] = 0.f;
    }
  }
  const float* s2 = red + kMlpRedSlab2Off + j;
  float p[4] = {0.f, 0.f, 0.f, 0.f};
  int r = q;
  for (; r + 12 < dw2_rows; r += 16)
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] += s2[(size_t)(r + 4 * k) * 65536];
  for (; r < dw2_rows; r += 4) p[0] += s2[(size_t)r * 65536];
  part2[q][e] = v + ((p[0] + p[1]) + (p[2] + p[3]));
  __syncthreads();
  if (q == 0) {
    const float t = (part2[0][e] + part2[1][e]) + (part2[2][e] + part2[3][e]);
    if (dW2 != nullptr && t != 0.f) dW2[j] += t;
  }
}

bool mlp_bwd8() {
  static const bool v = diag_env_int("WELLFLOW_MLP_BWD8", 1) != 0;  // A/B, WF_DIAG builds only
  return v;
}

int mlp2_train_grid(int B) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      return 256;
    return n;
  }();
  const int nchunks = (B + MF_ROWS_PUB - 1) / MF_ROWS_PUB;
  const int g = nchunks < cus ? nchunks : cus;
  return g < kMlpRedSlabRows ? g : kMlpRedSlabRows;
}

void launch_mlp2_reduce(float* red, int Fp, int B, float* loss_sum, float* db3, float* dw3, float* db1, float* db2,
                        float* dW1, float* dW2, hipStream_t s, int dw2_rows) {
  const int na = kMlpRedDW1;
  // the dW1 rows exist only when the 8-wave backward ran (the 4-wave one adds dW1 itself)
  const int slab_blocks = mlp_bwd8() ? (256 * Fp + 15) / 16 : 0;
  hipLaunchKernelGGL(mlp2_reduce_kernel, dim3(slab_blocks + (na + 255) / 256 + 65536 / 64), dim3(256), 0, s, red, Fp,
                     mlp2_train_grid(B), slab_blocks, loss_sum, db3, dw3, db1, db2, dW1, dW2,
                     dw2_rows < 0 ? 0 : (dw2_rows > kMlpRedSlab2Rows ? kMlpRedSlab2Rows : dw2_rows));
}


template <int KT1>  // layer-1 K steps of 32 features: 1 (Fp <= 32) or 2 (Fp <= 64)
__global__ __launch_bounds__(256, 1) void mlp2_fwd_kernel(
    const bf16_t* __restrict__ X, int Fp, const bf16_t* __restrict__ W1, const float* __restrict__ b1,
    const bf16_t* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ w3,
    const float* __restrict__ b3, const float* __restrict__ y, bf16_t* __restrict__ H1, bf16_t* __restrict__ H2,
    unsigned* __restrict__ M2, float* __restrict__ dw3, float* __restrict__ db3, float* __restrict__ pred,
    float* __restrict__ dy, float* __restrict__ loss_sum, float dy_scale, int B, const long long* __restrict__ rows,
    long nrows) {
  // rows != nullptr: batch row r is dataset row rows[r] of X / y (the resident dataset is read
  // in place, no gather kernel); H1 == nullptr: H1 is not stored (the training step's backward
  // recomputes it from X, inference never needs it)
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
  // the NEXT chunk's X row segment (thread: row t >> 2, chunk t & 3 (+4)) and target are loaded
  // right after this chunk's X tile is in LDS, so their latency hides behind this chunk's MFMAs
  // (one wave per SIMD: a load at the top of the chunk stalled every wave for its round trip)
  uint4 xv[KT1];
  float yv = 0.f;
  auto prefetch = [&](int ch) {
    const int r = threadIdx.x >> 2, gr = ch * MF_ROWS + r;
    const size_t dr = gr < B ? data_row(rows, gr, nrows) : 0;
#pragma unroll
    for (int k1 = 0; k1 < KT1; ++k1) {
      const int c = (threadIdx.x & 3) + 4 * k1;
      xv[k1] = (gr < B && 8 * c + 8 <= Fp) ? *reinterpret_cast<const uint4*>(X + dr * Fp + 8 * c)
                                           : make_uint4(0, 0, 0, 0);
    }
    const int ty = ch * MF_ROWS + (int)threadIdx.x;
    if (y != nullptr && threadIdx.x < MF_ROWS && ty < B) yv = y[data_row(rows, ty, nrows)];
  };
  if ((int)blockIdx.x < nchunks) prefetch(blockIdx.x);
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int row0 = ch * MF_ROWS;
    // ---- X chunk -> LDS, zero-padded to 32 * KT1 features
#pragma unroll
    for (int k1 = 0; k1 < KT1; ++k1)
      *reinterpret_cast<uint4*>(xs + xtile_off(threadIdx.x >> 2, (threadIdx.x & 3) + 4 * k1)) = xv[k1];
    const float ycur = yv;
    __syncthreads();
    if (ch + (int)gridDim.x < nchunks) prefetch(ch + gridDim.x);

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
    if (H1 != nullptr) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int idx = threadIdx.x + 256 * k, r = idx >> 5, c = idx & 31, gr = row0 + r;
        if (gr < B)
          *reinterpret_cast<uint4*>(H1 + (size_t)gr * MF_H + 8 * c) =
              *reinterpret_cast<const uint4*>(h1s + tile_off(r, 8 * c));
      }
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
          const float diff = p - ycur;
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
// The training-step forward (mask mode, neither H1 nor H2 stored) with 8 waves, two per SIMD:
// one wave's epilogue VALU / LDS traffic overlaps the other's MFMAs (the 4-wave kernel above
// holds 64 units per wave and leaves its SIMD idle through every epilogue and barrier).
//  * wave w owns hidden units [32w, 32w + 32) of both layers (W2 slice: 64 VGPRs).
//  * the H2 ReLU bitmask, the head gradients and the loss come straight from the layer-2
//    accumulators, with no H2 tile in LDS: a lane's bits (4 units x 2 M tiles of one row) are
//    OR-reduced over the row's 4 lane groups and stored as the wave's 32-bit mask word; dy of
//    the chunk's rows is rebuilt by every wave from the per-wave head partials, so
//    dw3 += H2^T dy accumulates in registers.
//  * three barriers per chunk (X staged, H1 tile complete, head partials complete); the
//    targets are double-buffered so the next chunk's staging never races this chunk's reads.
template <int KT1, int PR = 0>  // PR: s_setprio(1) around the layer-2 MFMA cluster (A/B)
__global__ __launch_bounds__(512, 1) void mlp2_fwd_train_kernel(
    const bf16_t* __restrict__ X, int Fp, const bf16_t* __restrict__ W1, const float* __restrict__ b1,
    const bf16_t* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ w3,
    const float* __restrict__ b3, const float* __restrict__ y, unsigned* __restrict__ M2, float* __restrict__ dw3,
    float* __restrict__ db3, float* __restrict__ pred, float* __restrict__ dy, float* __restrict__ loss_sum,
    float dy_scale, int B, const long long* __restrict__ rows, long nrows, int dbg, float* __restrict__ rscr) {
  // dbg (WELLFLOW_MLP_DBG, WF_DIAG builds only, timing only, wrong results): 1 = no epilogue
  // atomics, 2 = no W2 loads
  dbg &= kMlpDbgMask;
  // rscr != nullptr: the batch sums go to copy blockIdx % kMlpRedCopies of the spread-reduction scratch
  constexpr int NW = 8, MT = 2;  // waves; 16-unit M tiles per wave
  __shared__ __attribute__((aligned(16))) char xs[MF_ROWS * MF_XROW];
  __shared__ __attribute__((aligned(16))) char h1s[MF_ROWS * MF_H * 2];
  __shared__ __attribute__((aligned(16))) float red[MF_ROWS][NW];
  __shared__ float ys[2][MF_ROWS];
  __shared__ float lred[NW];

  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = threadIdx.x >> 6;
  const int u0 = wid * 16 * MT;
  bf16x8 w1f[KT1][MT], w2f[MT][8];
  float bias1[MT][4], bias2[MT][4], w3v[MT][4], dw3r[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int u = u0 + 16 * m + l15;
#pragma unroll
    for (int k1 = 0; k1 < KT1; ++k1) {
      const int f0 = 32 * k1 + 8 * g;
      w1f[k1][m] = f0 + 8 <= Fp ? *reinterpret_cast<const bf16x8*>(W1 + (size_t)u * Fp + f0)
                                : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
      w2f[m][kt] = (dbg & 2) ? bf16x8{0, 0, 0, 0, 0, 0, 0, 0}
                             : *reinterpret_cast<const bf16x8*>(W2 + (size_t)u * MF_H + 32 * kt + 8 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int uc = u0 + 16 * m + 4 * g + r;
      bias1[m][r] = b1[uc];
      bias2[m][r] = b2[uc];
      w3v[m][r] = w3[uc];
      dw3r[m][r] = 0.f;
    }
  }
  const float bias3 = b3[0];
  float lsum = 0.f, db3a = 0.f;

  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  // next chunk's inputs, loaded right after this chunk's are in LDS: threads 0..255 one X row
  // segment each (row t >> 2, chunk t & 3 (+4)), threads 256..319 one target
  uint4 xv[KT1];
  float yv = 0.f;
  auto prefetch = [&](int ch) {
    if (threadIdx.x < 256) {
      const int r = threadIdx.x >> 2, gr = ch * MF_ROWS + r;
      const size_t dr = gr < B ? data_row(rows, gr, nrows) : 0;
#pragma unroll
      for (int k1 = 0; k1 < KT1; ++k1) {
        const int c = (threadIdx.x & 3) + 4 * k1;
        xv[k1] = (gr < B && 8 * c + 8 <= Fp) ? *reinterpret_cast<const uint4*>(X + dr * Fp + 8 * c)
                                             : make_uint4(0, 0, 0, 0);
      }
    } else if (threadIdx.x < 256 + MF_ROWS) {
      const int ty = ch * MF_ROWS + (int)threadIdx.x - 256;
      yv = ty < B ? y[data_row(rows, ty, nrows)] : 0.f;
    }
  };
  if ((int)blockIdx.x < nchunks) prefetch(blockIdx.x);
  int par = 0;
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x, par ^= 1) {
    const int row0 = ch * MF_ROWS;
    if (threadIdx.x < 256) {
#pragma unroll
      for (int k1 = 0; k1 < KT1; ++k1)
        *reinterpret_cast<uint4*>(xs + xtile_off(threadIdx.x >> 2, (threadIdx.x & 3) + 4 * k1)) = xv[k1];
    } else if (threadIdx.x < 256 + MF_ROWS) {
      ys[par][threadIdx.x - 256] = yv;
    }
    __syncthreads();
    if (ch + (int)gridDim.x < nchunks) prefetch(ch + gridDim.x);

    // ---- layer 1: Z1^T (32 units x 64 rows per wave) = W1 x X^T
    f32x4 acc[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k1 = 0; k1 < KT1; ++k1)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(xs + xtile_off(16 * n + l15, 4 * k1 + g));
#pragma unroll
        for (int m = 0; m < MT; ++m)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[k1][m], xb, acc[m][n], 0, 0, 0);
      }
#pragma unroll
    for (int m = 0; m < MT; ++m)
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

    // ---- layer 2: Z2^T = W2 x H1^T, K = 256
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (PR & 1) __builtin_amdgcn_s_setprio(1);
    if constexpr ((PR & 2) != 0) {
      // A/B (WELLFLOW_MLP_DBG bit 2): H1 fragments double-buffered one k-step ahead
      bf16x8 hb[2][4];
#pragma unroll
      for (int n = 0; n < 4; ++n) hb[0][n] = *reinterpret_cast<const bf16x8*>(h1s + tile_off(16 * n + l15, 8 * g));
      static_for<0, 8>([&](auto kc) {
        constexpr int kt = decltype(kc)::value;
        if constexpr (kt + 1 < 8) {
#pragma unroll
          for (int n = 0; n < 4; ++n)
            hb[(kt + 1) & 1][n] = *reinterpret_cast<const bf16x8*>(h1s + tile_off(16 * n + l15, 32 * (kt + 1) + 8 * g));
        }
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[m][kt], hb[kt & 1][n], acc[m][n], 0, 0, 0);
      });
    } else {
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) {
        bf16x8 hb[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) hb[n] = *reinterpret_cast<const bf16x8*>(h1s + tile_off(16 * n + l15, 32 * kt + 8 * g));
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[m][kt], hb[n], acc[m][n], 0, 0, 0);
      }
    }
    if constexpr (PR & 1) __builtin_amdgcn_s_setprio(0);
    // ---- H2 = relu(Z2 + b2) rounded to bf16 (the values the backward's mask describes), kept
    // in acc; head partial sums and ReLU bits of rows 16n + l15
    float hp[4] = {0.f, 0.f, 0.f, 0.f};
    unsigned bits[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = bf2f(f2bf(fmaxf(acc[m][n][r] + bias2[m][r], 0.f)));
          acc[m][n][r] = v;
          hp[n] += v * w3v[m][r];
          if (v > 0.f) bits[n] |= 1u << (16 * m + 4 * g + r);
        }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      hp[n] += __shfl_xor(hp[n], 16, 64);
      hp[n] += __shfl_xor(hp[n], 32, 64);
      bits[n] |= (unsigned)__shfl_xor((int)bits[n], 16, 64);
      bits[n] |= (unsigned)__shfl_xor((int)bits[n], 32, 64);
    }
    if (g == 0) {
#pragma unroll
      for (int n = 0; n < 4; ++n) red[16 * n + l15][wid] = hp[n];
    }
    {  // lane group g stores the mask word of row 16g + l15 (units 32 wid .. 32 wid + 31)
      const unsigned bw = g == 0 ? bits[0] : g == 1 ? bits[1] : g == 2 ? bits[2] : bits[3];
      const int gr = row0 + 16 * g + l15;
      if (gr < B) M2[(size_t)gr * 8 + wid] = bw;
    }
    __syncthreads();

    // ---- prediction, dy and loss of rows 16n + l15 (every wave: its dw3 needs dy); wave 0
    // stores them, lane group g for row 16g + l15
    float dyn[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int r = 16 * n + l15, gr = row0 + r;
      const float4 pa = *reinterpret_cast<const float4*>(&red[r][0]);
      const float4 pb = *reinterpret_cast<const float4*>(&red[r][4]);
      const float p = ((pa.x + pa.y) + (pa.z + pa.w)) + ((pb.x + pb.y) + (pb.z + pb.w)) + bias3;
      dyn[n] = 0.f;
      if (gr < B) {
        const float diff = p - ys[par][r];
        dyn[n] = dy_scale * diff;
        if (wid == 0 && g == n) {
          if (pred != nullptr) pred[gr] = p;
          if (dy != nullptr) dy[gr] = dyn[n];
          lsum += diff * diff;
          db3a += dyn[n];
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int n = 0; n < 4; ++n) dw3r[m][r] += acc[m][n][r] * dyn[n];
  }
  if (dbg & 1) return;
  if (rscr != nullptr) {
    float* rb = rscr + (blockIdx.x & (kMlpRedCopies - 1)) * kMlpRedRow;
    if (loss_sum != nullptr) loss_sum = rb + kMlpRedLoss;
    dw3 = rb + kMlpRedDw3;
    db3 = rb + kMlpRedDb3;
  }
  if (loss_sum != nullptr) {
    const float t = block_sum<512>(lsum, lred);
    if (threadIdx.x == 0 && t != 0.f) atomicAdd(loss_sum, t);
  }
  // dw3: the 16 lanes l15 of a lane group hold the same 4 units (different rows)
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = dw3r[m][r];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if (l15 == 0 && v != 0.f) atomicAdd(dw3 + u0 + 16 * m + 4 * g + r, v);
    }
  const float t3 = block_sum<512>(db3a, lred);
  if (threadIdx.x == 0 && t3 != 0.f) atomicAdd(db3, t3);
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
    float* __restrict__ db2, float* __restrict__ dw3, float* __restrict__ db3, int B,
    const bf16_t* __restrict__ W1, const float* __restrict__ b1, const long long* __restrict__ rows, long nrows) {
  // H1 == nullptr (needs the fused dW1 path, Fp <= 32): H1 is RECOMPUTED from the X tile with
  // W1 / b1 in registers (8 extra MFMAs per wave and chunk) instead of being read back:
  // the forward no longer writes it (134 MB at B = 262144) and nothing reads it.
  // rows: dataset rows of X (as in the forward).
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
  const bool recompute = H1 == nullptr;
  // layer-1 weights for the recompute (lane = unit u0 + 16m + l15, features 8g..8g+7) and
  // biases (C rows: units u0 + 16m + 4g + r)
  bf16x8 w1f[4];
  float bias1[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    w1f[m] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) bias1[m][r] = 0.f;
    if (recompute) {
      const int u = u0 + 16 * m + l15;
      if (8 * g + 8 <= Fp) w1f[m] = *reinterpret_cast<const bf16x8*>(W1 + (size_t)u * Fp + 8 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) bias1[m][r] = b1[u0 + 16 * m + 4 * g + r];
    }
  }
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
        if (!recompute) h1v = *reinterpret_cast<const uint4*>(H1 + (size_t)gr * MF_H + 8 * c);
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
      if (!recompute) *reinterpret_cast<uint4*>(hs + tile_off(r, 8 * c)) = h1v;
      if (gr < B) *reinterpret_cast<uint4*>(dZ2 + (size_t)gr * MF_H + 8 * c) = zv;
    }
    if (fuse_dw1) {  // X chunk -> LDS, zero-padded to 32 features (as in the forward)
      const int r = threadIdx.x >> 2, xc = threadIdx.x & 3, gr = row0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (gr < B && 8 * xc + 8 <= Fp) {
        v = *reinterpret_cast<const uint4*>(X + data_row(rows, gr, nrows) * Fp + 8 * xc);
      }
      *reinterpret_cast<uint4*>(xs + xtile_off(r, xc)) = v;
    }
    __syncthreads();
    if (recompute) {
      // ---- H1 of this wave's 64 units (the forward's layer 1, bit-identical inputs): each lane
      // writes the 8 bytes the ReLU-mask phase below reads back (same lane, no barrier needed)
      f32x4 a1[4][4];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) a1[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(xs + xtile_off(16 * n + l15, g));
#pragma unroll
        for (int m = 0; m < 4; ++m) a1[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[m], xb, a1[m][n], 0, 0, 0);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          unsigned pk[2];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const float v0 = fmaxf(a1[m][n][2 * q] + bias1[m][2 * q], 0.f);
            const float v1 = fmaxf(a1[m][n][2 * q + 1] + bias1[m][2 * q + 1], 0.f);
            pk[q] = (unsigned)f2bf(v0) | ((unsigned)f2bf(v1) << 16);
          }
          *reinterpret_cast<uint2*>(hs + tile_off(16 * n + l15, u0 + 16 * m + 4 * g)) = make_uint2(pk[0], pk[1]);
        }
    }

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

// ----------------------------------------------------------------------------------------
// The training-step backward in its leanest form (mask mode + H1 recompute + fused dW1: the
// bench / job configuration, Fp <= 32): per 64-row chunk it reads only the H2 ReLU bits, dy and
// the X rows, and writes only dZ2. Same math as mlp2_bwd_kernel (that kernel's comments
// apply), organised for one wave per SIMD: the next chunk's bits, dy and X row segments are
// loaded right after the current chunk's tiles are in LDS, so their round trip hides behind
// this chunk's 152 MFMAs per wave instead of stalling every wave at the top of the chunk.
template <int NFT>
__global__ __launch_bounds__(256, 1) void mlp2_bwd_rc_kernel(
    const unsigned* __restrict__ M2, const float* __restrict__ dy, const float* __restrict__ w3,
    const bf16_t* __restrict__ W2, const bf16_t* __restrict__ X, int Fp, bf16_t* __restrict__ dZ2,
    float* __restrict__ dW1, float* __restrict__ db1, float* __restrict__ db2, int B,
    const bf16_t* __restrict__ W1, const float* __restrict__ b1, const long long* __restrict__ rows, long nrows) {
  __shared__ __attribute__((aligned(16))) char zs[MF_ROWS * MF_H * 2];  // dZ2 tile
  __shared__ __attribute__((aligned(16))) char hs[MF_ROWS * MF_H * 2];  // H1 tile -> dZ1 in place
  __shared__ __attribute__((aligned(16))) char xs[MF_ROWS * MF_XROW];   // X tile

  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = threadIdx.x >> 6;
  const int u0 = wid * 64;
  bf16x8 wt[4][8];  // W2^T (A operand: lane = input unit k = u0 + 16m + l15, K = output unit)
  bf16x8 w1f[4];    // W1 rows of this wave's units (recompute)
  float bias1[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int k = u0 + 16 * m + l15;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int j = 0; j < 8; ++j) wt[m][kt][j] = (short)W2[(size_t)(32 * kt + 8 * g + j) * MF_H + k];
    w1f[m] = 8 * g + 8 <= Fp ? *reinterpret_cast<const bf16x8*>(W1 + (size_t)k * Fp + 8 * g)
                             : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) bias1[m][r] = b1[u0 + 16 * m + 4 * g + r];
  }
  const int c = threadIdx.x & 31, rq = threadIdx.x >> 5;  // elementwise phase: units 8c.., rows rq + 8q
  float w3c[8], db2a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    w3c[e] = w3[8 * c + e];
    db2a[e] = 0.f;
  }
  float db1a[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) db1a[m][i] = 0.f;
  f32x4 dw1a[4][NFT];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int f = 0; f < NFT; ++f) dw1a[m][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int tq = (lane & 15) >> 2, tp = lane & 3;

  // prefetched inputs of one chunk: ReLU bits of units 8c..8c+7 and dy for rows rq + 8q, and
  // this thread's X row segment (row t >> 2, feature chunk t & 3)
  unsigned mb[8];
  float gyv[8];
  uint4 xv;
  auto prefetch = [&](int ch) {
    const int row0 = ch * MF_ROWS;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int gr = row0 + rq + 8 * q;
      mb[q] = gr < B ? M2[(size_t)gr * 8 + (c >> 2)] : 0u;
      gyv[q] = gr < B ? dy[gr] : 0.f;
    }
    const int xr = threadIdx.x >> 2, xc = threadIdx.x & 3, gr = row0 + xr;
    xv = (gr < B && 8 * xc + 8 <= Fp) ? *reinterpret_cast<const uint4*>(X + data_row(rows, gr, nrows) * Fp + 8 * xc)
                                      : make_uint4(0, 0, 0, 0);
  };
  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  if ((int)blockIdx.x < nchunks) prefetch(blockIdx.x);
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int row0 = ch * MF_ROWS;
    // ---- dZ2 = (dy w3^T) * [H2 > 0] -> LDS + HBM (dW2's operand); db2 partials
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = rq + 8 * q, gr = row0 + r;
      const unsigned bits = mb[q] >> (8 * (c & 3));
      unsigned zw[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        unsigned pk = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = 2 * p + h;
          const bf16_t zb = f2bf(((bits >> e) & 1u) ? gyv[q] * w3c[e] : 0.f);
          db2a[e] += bf2f(zb);
          pk |= (unsigned)zb << (16 * h);
        }
        zw[p] = pk;
      }
      const uint4 zv = make_uint4(zw[0], zw[1], zw[2], zw[3]);
      *reinterpret_cast<uint4*>(zs + tile_off(r, 8 * c)) = zv;
      if (gr < B) *reinterpret_cast<uint4*>(dZ2 + (size_t)gr * MF_H + 8 * c) = zv;
    }
    *reinterpret_cast<uint4*>(xs + xtile_off(threadIdx.x >> 2, threadIdx.x & 3)) = xv;
    __syncthreads();
    if (ch + (int)gridDim.x < nchunks) prefetch(ch + gridDim.x);

    // ---- H1 of this wave's units (bit-identical to the forward's layer 1) -> hs, own lanes only
    {
      f32x4 a1[4][4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(xs + xtile_off(16 * n + l15, g));
#pragma unroll
        for (int m = 0; m < 4; ++m)
          a1[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[m], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          unsigned pk[2];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const float v0 = fmaxf(a1[m][n][2 * q] + bias1[m][2 * q], 0.f);
            const float v1 = fmaxf(a1[m][n][2 * q + 1] + bias1[m][2 * q + 1], 0.f);
            pk[q] = (unsigned)f2bf(v0) | ((unsigned)f2bf(v1) << 16);
          }
          *reinterpret_cast<uint2*>(hs + tile_off(16 * n + l15, u0 + 16 * m + 4 * g)) = make_uint2(pk[0], pk[1]);
        }
    }
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
    // ---- dZ1 = dH1 * [H1 > 0] into the same 8 bytes of hs; db1 partials
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int r = 16 * n + l15;
        uint2* pp = reinterpret_cast<uint2*>(hs + tile_off(r, u0 + 16 * m + 4 * g));
        const uint2 hv = *pp;
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
        *pp = make_uint2(ow[0], ow[1]);
      }
    __syncthreads();
    // ---- dW1^T slice (64 units x Fp per wave) += dZ1^T X over the chunk's rows
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[NFT];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 32 * kk + 8 * g + 4 * h + tq;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(hs + tile_off(r, u0 + 16 * m + 4 * tp)));
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
  }
  // ---- reductions (as mlp2_bwd_kernel)
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
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int f = 0; f < NFT; ++f) {
      const int ft = l15 + 16 * f;
      if (ft < Fp)
#pragma unroll
        for (int i = 0; i < 4; ++i) atomicAdd(dW1 + (size_t)(u0 + 16 * m + 4 * g + i) * Fp + ft, dw1a[m][f][i]);
    }
  float* sd = reinterpret_cast<float*>(zs);
#pragma unroll
  for (int e = 0; e < 8; ++e) sd[rq * MF_H + 8 * c + e] = db2a[e];
  __syncthreads();
  float s2 = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) s2 += sd[q * MF_H + threadIdx.x];
  if (s2 != 0.f) atomicAdd(db2 + threadIdx.x, s2);
}

// ----------------------------------------------------------------------------------------
// mlp2_bwd_rc_kernel with 8 waves, two per SIMD (wave w owns input units [32w, 32w + 32):
// W2^T slice 64 VGPRs), so one wave's dZ2 / dZ1 elementwise work and LDS traffic overlaps the
// other's MFMAs. The dZ2 and X tiles are double-buffered and the H1 / dZ1 tile is wave-private
// (every wave reads back only its own units), so a chunk needs ONE workgroup barrier: the
// next chunk's staging writes the other buffer, whose last readers passed this barrier.
template <int NFT, int PR = 0>  // PR: s_setprio(1) around the dH1 MFMA cluster (A/B)
__global__ __launch_bounds__(512, 1) void mlp2_bwd_rc8_kernel(
    const unsigned* __restrict__ M2, const float* __restrict__ dy, const float* __restrict__ w3,
    const bf16_t* __restrict__ W2, const bf16_t* __restrict__ X, int Fp, bf16_t* __restrict__ dZ2,
    float* __restrict__ dW1, float* __restrict__ db1, float* __restrict__ db2, int B,
    const bf16_t* __restrict__ W1, const float* __restrict__ b1, const long long* __restrict__ rows, long nrows,
    int dbg, float* __restrict__ red) {
  // red != nullptr: db1, db2 go to copy blockIdx % kMlpRedCopies of the spread-reduction scratch, dW1 to this workgroup's row
  // dbg (WELLFLOW_MLP_DBG, WF_DIAG builds only, timing only, wrong results): 1 = no epilogue
  // atomics, 2 = no W2^T gather
  dbg &= kMlpDbgMask;
  constexpr int MT = 2, ZB = MF_ROWS * MF_H * 2, XB = MF_ROWS * MF_XROW;
  __shared__ __attribute__((aligned(16))) char zs[2 * ZB];  // dZ2 tiles (double-buffered)
  __shared__ __attribute__((aligned(16))) char hs[ZB];      // H1 -> dZ1 in place (wave-private units)
  __shared__ __attribute__((aligned(16))) char xs[2 * XB];  // X tiles (double-buffered)

  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = threadIdx.x >> 6;
  const int u0 = wid * 16 * MT;
  bf16x8 wt[MT][8];  // W2^T (A operand: lane = input unit k = u0 + 16m + l15, K = output unit)
  bf16x8 w1f[MT];    // W1 rows of this wave's units (recompute)
  float bias1[MT][4], db1a[MT][4];
  f32x4 dw1a[MT][NFT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int k = u0 + 16 * m + l15;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int j = 0; j < 8; ++j) wt[m][kt][j] = (dbg & 2) ? (short)0 : (short)W2[(size_t)(32 * kt + 8 * g + j) * MF_H + k];
    w1f[m] = 8 * g + 8 <= Fp ? *reinterpret_cast<const bf16x8*>(W1 + (size_t)k * Fp + 8 * g)
                             : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bias1[m][r] = b1[u0 + 16 * m + 4 * g + r];
      db1a[m][r] = 0.f;
    }
#pragma unroll
    for (int f = 0; f < NFT; ++f) dw1a[m][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int c = threadIdx.x & 31, rq = threadIdx.x >> 5;  // elementwise phase: units 8c.., rows rq + 16q
  float w3c[8], db2a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    w3c[e] = w3[8 * c + e];
    db2a[e] = 0.f;
  }
  const int tq = (lane & 15) >> 2, tp = lane & 3;

  unsigned mb[4];
  float gyv[4];
  uint4 xv = make_uint4(0, 0, 0, 0);
  auto prefetch = [&](int ch) {
    const int row0 = ch * MF_ROWS;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int gr = row0 + rq + 16 * q;
      mb[q] = gr < B ? M2[(size_t)gr * 8 + (c >> 2)] : 0u;
      gyv[q] = gr < B ? dy[gr] : 0.f;
    }
    if (threadIdx.x < 256) {
      const int xr = threadIdx.x >> 2, xc = threadIdx.x & 3, gr = row0 + xr;
      xv = (gr < B && 8 * xc + 8 <= Fp) ? *reinterpret_cast<const uint4*>(X + data_row(rows, gr, nrows) * Fp + 8 * xc)
                                        : make_uint4(0, 0, 0, 0);
    }
  };
  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  if ((int)blockIdx.x < nchunks) prefetch(blockIdx.x);
  int par = 0;
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x, par ^= 1) {
    const int row0 = ch * MF_ROWS;
    char* zt = zs + par * ZB;
    char* xt = xs + par * XB;
    // ---- dZ2 = (dy w3^T) * [H2 > 0] -> LDS + HBM (dW2's operand); db2 partials
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = rq + 16 * q, gr = row0 + r;
      const int bits = (int)(mb[q] >> (8 * (c & 3)));
      const int gyb = __float_as_int(gyv[q]);
      unsigned zw[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        // bit e sign-extended (v_bfe_i32) masks dy: t = [H2 > 0] dy, two VALU ops per element
        // instead of shift / and / compare / select. db2 = w3 * sum t is accumulated in fp32
        // before the bf16 rounding of dZ2 (the reduction's w3 factor is applied once, below)
        const float t0 = __int_as_float(__builtin_amdgcn_sbfe(bits, 2 * p, 1) & gyb);
        const float t1 = __int_as_float(__builtin_amdgcn_sbfe(bits, 2 * p + 1, 1) & gyb);
        db2a[2 * p] += t0;
        db2a[2 * p + 1] += t1;
        zw[p] = pk_bf16(t0 * w3c[2 * p], t1 * w3c[2 * p + 1]);
      }
      const uint4 zv = make_uint4(zw[0], zw[1], zw[2], zw[3]);
      *reinterpret_cast<uint4*>(zt + tile_off(r, 8 * c)) = zv;
      if (gr < B) *reinterpret_cast<uint4*>(dZ2 + (size_t)gr * MF_H + 8 * c) = zv;
    }
    if (threadIdx.x < 256) *reinterpret_cast<uint4*>(xt + xtile_off(threadIdx.x >> 2, threadIdx.x & 3)) = xv;
    __syncthreads();
    if (ch + (int)gridDim.x < nchunks) prefetch(ch + gridDim.x);

    // ---- H1 of this wave's units (bit-identical to the forward's layer 1) -> hs
    {
      f32x4 a1[MT][4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(xt + xtile_off(16 * n + l15, g));
#pragma unroll
        for (int m = 0; m < MT; ++m)
          a1[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[m], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          unsigned pk[2];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const float v0 = fmaxf(a1[m][n][2 * q] + bias1[m][2 * q], 0.f);
            const float v1 = fmaxf(a1[m][n][2 * q + 1] + bias1[m][2 * q + 1], 0.f);
            pk[q] = (unsigned)f2bf(v0) | ((unsigned)f2bf(v1) << 16);
          }
          *reinterpret_cast<uint2*>(hs + tile_off(16 * n + l15, u0 + 16 * m + 4 * g)) = make_uint2(pk[0], pk[1]);
        }
    }
    // ---- dH1^T (32 k x 64 rows per wave) = W2^T x dZ2^T, K = 256
    f32x4 acc[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (PR) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      bf16x8 zb[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) zb[n] = *reinterpret_cast<const bf16x8*>(zt + tile_off(16 * n + l15, 32 * kt + 8 * g));
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wt[m][kt], zb[n], acc[m][n], 0, 0, 0);
    }
    if constexpr (PR) __builtin_amdgcn_s_setprio(0);
    // ---- dZ1 = dH1 * [H1 > 0] into the same 8 bytes of hs; db1 partials
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int r = 16 * n + l15;
        uint2* pp = reinterpret_cast<uint2*>(hs + tile_off(r, u0 + 16 * m + 4 * g));
        const uint2 hv = *pp;
        const bool rok = row0 + r < B;
        const int hw2[2] = {rok ? (int)hv.x : 0, rok ? (int)hv.y : 0};
        unsigned ow[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          // H1 >= 0 (relu), so H1 > 0 <=> the bf16 half is > 0 as a signed 16-bit integer (-0 is
          // not): low half via the sign of (w << 16), high half as w > 0xFFFF signed
          const bool on0 = (hw2[q] << 16) > 0, on1 = hw2[q] > 0xFFFF;
          const float t0 = on0 ? acc[m][n][2 * q] : 0.f, t1 = on1 ? acc[m][n][2 * q + 1] : 0.f;
          db1a[m][2 * q] += t0;  // fp32 before the bf16 rounding of dZ1
          db1a[m][2 * q + 1] += t1;
          ow[q] = pk_bf16(t0, t1);
        }
        *pp = make_uint2(ow[0], ow[1]);
      }
    // the dW1 fragments below read other lanes' dZ1 (same wave): complete the writes first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // ---- dW1^T slice (32 units x Fp per wave) += dZ1^T X over the chunk's rows
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MT], bfr[NFT];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 32 * kk + 8 * g + 4 * h + tq;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(hs + tile_off(r, u0 + 16 * m + 4 * tp)));
#pragma unroll
          for (int e = 0; e < 4; ++e) af[m][4 * h + e] = v[e];
        }
#pragma unroll
        for (int f = 0; f < NFT; ++f) {
          const int f0 = 16 * f + 4 * tp;
          const bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(xt + xtile_off(r, f0 >> 3) + ((f0 & 7) << 1)));
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[f][4 * h + e] = v[e];
        }
      }
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int f = 0; f < NFT; ++f)
          dw1a[m][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[f], dw1a[m][f], 0, 0, 0);
    }
    // hs is rewritten by this wave's next H1 recompute: its dW1 reads must be complete
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  // ---- reductions
  if (dbg & 1) return;
  float* slab = nullptr;  // this workgroup's dW1 row (plain stores, summed by mlp2_reduce)
  if (red != nullptr) {
    float* rb = red + (blockIdx.x & (kMlpRedCopies - 1)) * kMlpRedRow;
    db1 = rb + kMlpRedDb1;
    db2 = rb + kMlpRedDb2;
    slab = red + kMlpRedSlabOff + (size_t)blockIdx.x * kMlpRedSlabRow;
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = db1a[m][i];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if (l15 == 0 && v != 0.f) atomicAdd(db1 + u0 + 16 * m + 4 * g + i, v);
    }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int f = 0; f < NFT; ++f) {
      const int ft = l15 + 16 * f;
      if (ft < Fp) {
        if (slab != nullptr) {
#pragma unroll
          for (int i = 0; i < 4; ++i) slab[(u0 + 16 * m + 4 * g + i) * Fp + ft] = dw1a[m][f][i];
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) atomicAdd(dW1 + (size_t)(u0 + 16 * m + 4 * g + i) * Fp + ft, dw1a[m][f][i]);
        }
      }
    }
  __syncthreads();  // the last chunk's dZ2 tile reads are done before zs becomes the db2 scratch
  float* sd = reinterpret_cast<float*>(zs);
#pragma unroll
  for (int e = 0; e < 8; ++e) sd[rq * MF_H + 8 * c + e] = db2a[e] * w3c[e];
  __syncthreads();
  if (threadIdx.x < MF_H) {
    float s2 = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) s2 += sd[q * MF_H + threadIdx.x];
    if (s2 != 0.f) atomicAdd(db2 + threadIdx.x, s2);
  }
}

// ----------------------------------------------------------------------------------------
// dW2 += dZ2^T H1 with H1 = relu(X W1^T + b1) RECOMPUTED per 64-row chunk instead of being
// stored by the forward and re-read here (the generic split-K GEMM read H1 [B][256] twice:
// 268 MB at B = 262144). Per chunk a workgroup streams its dZ2 columns (MN-contiguous image,
// LDS-DMA) and the 64 X rows (LDS-DMA per-lane gather, so `rows` indirection costs nothing),
// rebuilds its 128 H1 units from the X tile with W1 in registers (8 MFMAs per wave), writes
// them straight into the MN-contiguous image the dW MFMAs read (gemm_core.h swizzle), and
// accumulates the 128 x 128 output tile in registers (32 MFMAs per wave per chunk).
//  * grid = 4 output tiles x nsplit row ranges (one workgroup per CU at nsplit = 64); the 4
//    tiles of one row range are consecutive logical ids, so xcd_remap puts them on one XCD
//    and the second reader of each dZ2 chunk hits L2.
//  * 3-stage ring of {dZ2 16 KB, X 4 KB}, two barriers per chunk, counted vmcnt.
//  * X padding: features >= Fp are multiplied by zero W1 columns; their lanes DMA a valid
//    chunk of the same row (finite values), never out-of-bounds memory.
constexpr int DW2_STAGES = 4;
constexpr int DW2_MAX_ROWS = 8192;  // rows per workgroup (the LDS row-id table)
// NW = 4: waves 2(M) x 2(N) of 64x64, each rebuilding 32 H1 units; NW = 8 (default): two waves
// per SIMD, 2(M) x 4(N) of 64x32, 16 H1 units each, so one wave's H1 rebuild (VALU) and
// fragment reads overlap the other's MFMAs. The X tile is 4 one-KiB pieces, issued by waves
// 0-3: with 8 waves the DMA count per chunk differs by wave (dma_wait below).
template <int NW, int PR = 0>  // PR: s_setprio(1) around each MFMA cluster (A/B)
__global__ __launch_bounds__(64 * NW, 1) void mlp2_dw2_kernel(const bf16_t* __restrict__ dZ2, const bf16_t* __restrict__ X,
                                                              int Fp, const long long* __restrict__ rows, long nrows,
                                                              const bf16_t* __restrict__ W1, const float* __restrict__ b1,
                                                              int kchunk, float* __restrict__ dW2, float* __restrict__ red,
                                                              int mlp_dbg_dev) {
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  mlp_dbg_dev &= kMlpDbgMask;  // WF_DIAG builds only
  constexpr int NT = 64 * NW, BM = 128, BN = 128, MTR = 128 / (16 * NW);  // H1 unit tiles per wave
  using C = GemmCfg<BM, BN, MN_CONTIG, MN_CONTIG, 2, NW / 2>;
  using QA = GldsTile<BM, MN_CONTIG, NT>;
  constexpr int ABYTES = QA::BYTES;           // 16 KB: [64 rows][128 units]
  constexpr int XBYTES = MF_ROWS * 64;        // 4 KB: [64 rows][4 x 16-B feature chunks]
  constexpr int SLOT = ABYTES + XBYTES;
  constexpr int HIMG = BN * 64 * 2;           // one H1 image [64 rows][128 units], 16 KB
  constexpr int HOFF = DW2_STAGES * SLOT;     // two H1 images (chunk c read while c + 1 is built)
  constexpr int LPT_X = QA::PER_WAVE + 1;     // DMA instructions per chunk: waves 0-3 (A + X)
  constexpr int LPT_A = QA::PER_WAVE;         //   waves 4-7 (A only)
  constexpr int ROFF = HOFF + 2 * HIMG;       // dataset row ids of the range (int32), read from
                                              // LDS: a global index load would join the vmcnt
                                              // queue and drain the DMA prefetch
  __shared__ __attribute__((aligned(16))) char smem[ROFF + DW2_MAX_ROWS * 4];
  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / (NW / 2), wn = wid % (NW / 2);
  const bool xw = wid < 4;  // this wave DMAs one X piece per chunk
  // wait until at most n chunks' DMA of this wave are in flight (counts differ by wave)
  auto dma_wait = [&](auto nc) {
    constexpr int n = decltype(nc)::value;
    if (NW == 4 || xw)
      wait_vmcnt<n * LPT_X>();
    else
      wait_vmcnt<n * LPT_A>();
  };
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L >> 2, t = L & 3;
  const int m0 = (t >> 1) * BM, n0 = (t & 1) * BN;
  const int kbeg = split * kchunk;
  const int nk = kchunk / MF_ROWS;
  int* ridx = reinterpret_cast<int*>(smem + ROFF);
  if (rows != nullptr) {
    for (int i = threadIdx.x; i < kchunk; i += NT) ridx[i] = (int)data_row(rows, kbeg + i, nrows);
    __syncthreads();
  }

  // recompute operands: this wave builds H1 units n0 + 16 MTR wid .. (MTR tiles of 16)
  bf16x8 w1f[MTR];
  float bias1[MTR][4];
#pragma unroll
  for (int mt = 0; mt < MTR; ++mt) {
    const int u = n0 + 16 * (MTR * wid + mt) + l15;
    w1f[mt] = 8 * g + 8 <= Fp ? *reinterpret_cast<const bf16x8*>(W1 + (size_t)u * Fp + 8 * g)
                              : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) bias1[mt][r] = b1[n0 + 16 * (MTR * wid + mt) + 4 * g + r];
  }
  // X gather (waves 0-3): lane -> tile row 16 wid + (lane >> 2), LDS chunk slot lane & 3
  // holding feature chunk (slot ^ ((row >> 2) & 3)) (conflict-free fragment reads below)
  const int xrow = 16 * (wid & 3) + (lane >> 2);
  int xc = (lane & 3) ^ ((xrow >> 2) & 3);
  if (8 * xc + 8 > Fp) xc = 0;  // padding: any finite chunk of the same row (W1 there is 0)
  auto issue = [&](int c, int slot) {
    char* st = smem + slot * SLOT;
    QA::issue(dZ2, MF_H, m0, kbeg + c * MF_ROWS, st, wid, lane);
    if (NW == 4 || xw) {
      const size_t xr = rows != nullptr ? (size_t)ridx[c * MF_ROWS + xrow] : (size_t)(kbeg + c * MF_ROWS + xrow);
      __builtin_amdgcn_global_load_lds((const void*)(X + xr * Fp + 8 * xc),
                                       (lds_void*)(st + ABYTES + (wid & 3) * 1024), 16, 0, 0);
    }
  };
  using SW = MnSwz<BN>;
  // H1 = relu(X W1^T + b1) of chunk c (X in ring slot) -> H1 image `img` (MN-contiguous operand:
  // element (k = chunk row, n) of the dW GEMM's B operand)
  auto recompute = [&](int slot, int img) {
    const char* st = smem + slot * SLOT;
    f32x4 a1[MTR][4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int r = 16 * nt + l15;
      const bf16x8 xb = *reinterpret_cast<const bf16x8*>(st + ABYTES + r * 64 + ((g ^ ((r >> 2) & 3)) << 4));
#pragma unroll
      for (int mt = 0; mt < MTR; ++mt)
        a1[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[mt], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    const unsigned hbase = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)(smem + HOFF + img * HIMG));
#pragma unroll
    for (int mt = 0; mt < MTR; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int r = 16 * nt + l15;
        unsigned pk[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float v0 = fmaxf(a1[mt][nt][2 * q] + bias1[mt][2 * q], 0.f);
          const float v1 = fmaxf(a1[mt][nt][2 * q + 1] + bias1[mt][2 * q + 1], 0.f);
          pk[q] = (unsigned)f2bf(v0) | ((unsigned)f2bf(v1) << 16);
        }
        const unsigned off = r * (BN * 2) + (SW::pos(MTR * wid + mt, SW::hk(r)) << 5) + 8 * g;
        // LDS writes in asm: compiler-visible ones get a vmcnt(0) guard behind the LDS-DMA
        asm volatile("ds_write_b64 %0, %1" ::"v"(hbase + off), "v"(make_uint2(pk[0], pk[1])) : "memory");
      }
  };
  FragReader<BM, MN_CONTIG, C::WTM> fa;
  FragReader<BN, MN_CONTIG, C::WTN> fb;
  fa.init(wm * C::WTM, lane);
  fb.init(wn * C::WTN, lane);
  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: chunks 0..2 in flight, H1 of chunk 0 built
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  if (nk > 2) issue(2, 2);
  if (nk > 2) dma_wait(std::integral_constant<int, 2>{});
  else if (nk > 1) dma_wait(std::integral_constant<int, 1>{});
  else dma_wait(std::integral_constant<int, 0>{});
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  recompute(0, 0);

  // chunk c: [wait chunk c+1's DMA, barrier] issue c+3 | build H1(c+1) | dW MFMAs of c
  auto body = [&](int c, auto sc) {
    constexpr int S = decltype(sc)::value;  // == c % 4 (ring slot of chunk c); H1 image c & 1
    if (c + 2 < nk) dma_wait(std::integral_constant<int, 1>{});
    else dma_wait(std::integral_constant<int, 0>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's H1 image writes
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + 3 < nk) issue(c + 3, (S + 3) % DW2_STAGES);
    if (c + 1 < nk) recompute((S + 1) % DW2_STAGES, (S + 1) & 1);
    static_for<0, 2>([&](auto kc) {
      constexpr int KK = decltype(kc)::value;
      bf16x8 a[C::TM], b[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i) a[i] = fa.template frag<KK, S * SLOT>(smem, i);
#pragma unroll
      for (int j = 0; j < C::TN; ++j) b[j] = fb.template frag<KK, HOFF + (S & 1) * HIMG>(smem, j);
      if constexpr (PR) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      if constexpr (PR) __builtin_amdgcn_s_setprio(0);
    });
  };
  int c = 0;
  for (; c + 4 <= nk; c += 4) {
    body(c, std::integral_constant<int, 0>{});
    body(c + 1, std::integral_constant<int, 1>{});
    body(c + 2, std::integral_constant<int, 2>{});
    body(c + 3, std::integral_constant<int, 3>{});
  }
  if (c < nk) body(c, std::integral_constant<int, 0>{});
  if (c + 1 < nk) body(c + 1, std::integral_constant<int, 1>{});
  if (c + 2 < nk) body(c + 2, std::integral_constant<int, 2>{});
  const AccCoord<C> cc(m0, n0);
  // red != nullptr: copy split % 4 of the spread-reduction scratch (64 -> 16 adders per address)
  if (red != nullptr) dW2 = red + kMlpRedCopies * kMlpRedRow + (split & (kMlpRedCopies2 - 1)) * 65536;
  if (mlp_dbg_dev & 1) return;  // timing only (WELLFLOW_MLP_DBG): no epilogue atomics
#pragma unroll
  for (int j = 0; j < C::TN; ++j)
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(dW2 + (size_t)cc.row(i, r) * MF_H + cc.col(j), acc[i][j][r]);
}

// dW2 [256][256] fp32 (atomics: zeroed or accumulating) from dZ2 [B][256], X rows (rows), W1, b1.
// Needs B % 64 == 0 and Fp <= 32 (one K = 32 layer-1 step); false = not covered.
bool launch_mlp2_dw2(const bf16_t* dZ2, const bf16_t* X, int Fp, const long long* rows, long nrows, const bf16_t* W1,
                     const float* b1, int B, int nsplit, float* dW2, hipStream_t s, float* red) {
  if (B <= 0 || B % MF_ROWS != 0 || Fp > 32 || Fp % 8 != 0) return false;
  const int chunks = B / MF_ROWS;
  if (nsplit < 1) nsplit = 1;
  while (nsplit > 1 && chunks % nsplit != 0) --nsplit;
  const int kchunk = (chunks / nsplit) * MF_ROWS;
  if (rows != nullptr && kchunk > DW2_MAX_ROWS) return false;
  static const bool dw2_8 = diag_env_int("WELLFLOW_MLP_DW2_8", 1) != 0;  // A/B, WF_DIAG builds only
  if (dw2_8 && (mlp_prio() & 4))
    hipLaunchKernelGGL((mlp2_dw2_kernel<8, 1>), dim3(4 * nsplit), dim3(512), 0, s, dZ2, X, Fp, rows, nrows, W1, b1, kchunk,
                       dW2, red, mlp_dbg());
  else if (dw2_8)
    hipLaunchKernelGGL(mlp2_dw2_kernel<8>, dim3(4 * nsplit), dim3(512), 0, s, dZ2, X, Fp, rows, nrows, W1, b1, kchunk,
                       dW2, red, mlp_dbg());
  else
    hipLaunchKernelGGL(mlp2_dw2_kernel<4>, dim3(4 * nsplit), dim3(256), 0, s, dZ2, X, Fp, rows, nrows, W1, b1, kchunk,
                       dW2, red, mlp_dbg());
  return true;
}

bool launch_mlp2_bwd(const bf16_t* H1, const bf16_t* H2, const unsigned* M2, const float* dy, const float* w3, const bf16_t* W2,
                     const bf16_t* X, int Fp, bf16_t* dZ1, bf16_t* dZ2, float* dW1, float* db1, float* db2,
                     float* dw3, float* db3, int B, const bf16_t* W1, const float* b1, const long long* rows,
                     long nrows, hipStream_t s, float* red) {
  if (B <= 0 || (dW1 != nullptr && (X == nullptr || Fp > 32 || Fp % 8 != 0))) return false;
  if (H1 == nullptr && (dW1 == nullptr || W1 == nullptr || b1 == nullptr)) return false;  // recompute needs the X tile
  if (rows != nullptr && dW1 == nullptr) return false;  // X is read only by the fused dW1 path
  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  // with the spread scratch, the grid is the one mlp2_reduce sums the dW1 rows of
  const int grid = red != nullptr ? mlp2_train_grid(B) : (nchunks < cus ? nchunks : cus);
  if (H1 == nullptr && M2 != nullptr && dW1 != nullptr) {  // the training step's configuration
    if (mlp_bwd8()) {
      if (Fp <= 16 && (mlp_prio() & 2))
        hipLaunchKernelGGL((mlp2_bwd_rc8_kernel<1, 1>), dim3(grid), dim3(512), 0, s, M2, dy, w3, W2, X, Fp, dZ2, dW1, db1,
                           db2, B, W1, b1, rows, nrows, mlp_dbg(), red);
      else if (Fp <= 16)
        hipLaunchKernelGGL(mlp2_bwd_rc8_kernel<1>, dim3(grid), dim3(512), 0, s, M2, dy, w3, W2, X, Fp, dZ2, dW1, db1,
                           db2, B, W1, b1, rows, nrows, mlp_dbg(), red);
      else
        hipLaunchKernelGGL(mlp2_bwd_rc8_kernel<2>, dim3(grid), dim3(512), 0, s, M2, dy, w3, W2, X, Fp, dZ2, dW1, db1,
                           db2, B, W1, b1, rows, nrows, mlp_dbg(), red);
      return true;
    }
    if (Fp <= 16)
      hipLaunchKernelGGL(mlp2_bwd_rc_kernel<1>, dim3(grid), dim3(256), 0, s, M2, dy, w3, W2, X, Fp, dZ2, dW1, db1, db2,
                         B, W1, b1, rows, nrows);
    else
      hipLaunchKernelGGL(mlp2_bwd_rc_kernel<2>, dim3(grid), dim3(256), 0, s, M2, dy, w3, W2, X, Fp, dZ2, dW1, db1, db2,
                         B, W1, b1, rows, nrows);
    return true;
  }
  if (Fp <= 16)
    hipLaunchKernelGGL(mlp2_bwd_kernel<1>, dim3(grid), dim3(256), 0, s, H1, H2, M2, dy, w3, W2, X, Fp, dZ1, dZ2, dW1,
                       db1, db2, dw3, db3, B, W1, b1, rows, nrows);
  else
    hipLaunchKernelGGL(mlp2_bwd_kernel<2>, dim3(grid), dim3(256), 0, s, H1, H2, M2, dy, w3, W2, X, Fp, dZ1, dZ2, dW1,
                       db1, db2, dw3, db3, B, W1, b1, rows, nrows);
  return true;
}

bool launch_mlp2_fwd(const bf16_t* X, int Fp, const bf16_t* W1, const float* b1, const bf16_t* W2, const float* b2,
                     const float* w3, const float* b3, const float* y, bf16_t* H1, bf16_t* H2, unsigned* M2,
                     float* dw3, float* db3, float* pred, float* dy, float* loss_sum, float dy_scale, int B,
                     const long long* rows, long nrows, hipStream_t s, float* red) {
  if (Fp > 64 || Fp % 8 != 0 || B <= 0) return false;
  if (M2 != nullptr && (y == nullptr || dw3 == nullptr || db3 == nullptr)) return false;
  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int grid = nchunks < cus ? nchunks : cus;
  static const bool fwd8 = diag_env_int("WELLFLOW_MLP_FWD8", 1) != 0;  // A/B, WF_DIAG builds only
  if (fwd8 && M2 != nullptr && H1 == nullptr) {  // the training step (mask mode never writes H2)
    if (Fp <= 32 && (mlp_prio() & 1))
      hipLaunchKernelGGL((mlp2_fwd_train_kernel<1, 1>), dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y,
                         M2, dw3, db3, pred, dy, loss_sum, dy_scale, B, rows, nrows, mlp_dbg(), red);
    else if (Fp <= 32 && (mlp_dbg() & 4))
      hipLaunchKernelGGL((mlp2_fwd_train_kernel<1, 2>), dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y,
                         M2, dw3, db3, pred, dy, loss_sum, dy_scale, B, rows, nrows, mlp_dbg(), red);
    else if (Fp <= 32)
      hipLaunchKernelGGL(mlp2_fwd_train_kernel<1>, dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y, M2,
                         dw3, db3, pred, dy, loss_sum, dy_scale, B, rows, nrows, mlp_dbg(), red);
    else
      hipLaunchKernelGGL(mlp2_fwd_train_kernel<2>, dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y, M2,
                         dw3, db3, pred, dy, loss_sum, dy_scale, B, rows, nrows, mlp_dbg(), red);
    return true;
  }
  if (Fp <= 32)
    hipLaunchKernelGGL(mlp2_fwd_kernel<1>, dim3(grid), dim3(256), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y, H1, H2,
                       M2, dw3, db3, pred, dy, loss_sum, dy_scale, B, rows, nrows);
  else
    hipLaunchKernelGGL(mlp2_fwd_kernel<2>, dim3(grid), dim3(256), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y, H1, H2,
                       M2, dw3, db3, pred, dy, loss_sum, dy_scale, B, rows, nrows);
  return true;
}

}  // namespace wf
