// wellflow — regression head, losses, fused optimizers, casts (gfx950).
//
// K6 (mae_clip fwd+bwd in one kernel), K8 (SGD-Nesterov with Keras-0.x
// time decay, one launch over the flat buffer), K15 (regression head), K16 (MSE fwd+bwd,
// wave64 shuffle reduction + one atomic per workgroup), K17 (fused Adam over the flat
// fp32 master buffer, float4-vectorised), K18 (casts).
#include <cstdlib>

#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "lstm_layout.h"

namespace wf {

// ---------------------------------------------------------------- regression head (N=1)
// Row groups of LPR lanes (LPR = Hd/8 rounded up to a power of two, <= 64) each own one
// row: a lane loads 16 B (8 bf16) of it, the group reduces with xor-shuffles. The loss is
// block-reduced and added with ONE atomic per workgroup (same-address atomics from every
// workgroup were 33% of the MLP step before).
template <int LPR>
__global__ __launch_bounds__(256) void head_fwd_kernel(const bf16_t* __restrict__ Hm, long ldh,
                                                       int B, int Hd, const float* __restrict__ w,
                                                       const float* __restrict__ b0,
                                                       const float* __restrict__ target,
                                                       float* __restrict__ pred,
                                                       float* __restrict__ dy,
                                                       float* __restrict__ loss_sum,
                                                       float dy_scale) {
  __shared__ float red[4];
  constexpr int RPB = 256 / LPR;  // rows per block pass
  const int sub = threadIdx.x % LPR, grp = threadIdx.x / LPR;
  const float bias = b0[0];
  float lsum = 0.f;
  for (int rb = blockIdx.x * RPB; rb < B; rb += gridDim.x * RPB) {
    const int b = rb + grp;
    float acc = 0.f;
    if (b < B) {
      const bf16_t* row = Hm + (size_t)b * ldh;
      for (int k = sub * 8; k < Hd; k += LPR * 8) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(row + k);
        const float4 w0 = *reinterpret_cast<const float4*>(w + k);
        const float4 w1 = *reinterpret_cast<const float4*>(w + k + 4);
        acc += bf2f((bf16_t)v[0]) * w0.x + bf2f((bf16_t)v[1]) * w0.y + bf2f((bf16_t)v[2]) * w0.z +
               bf2f((bf16_t)v[3]) * w0.w + bf2f((bf16_t)v[4]) * w1.x + bf2f((bf16_t)v[5]) * w1.y +
               bf2f((bf16_t)v[6]) * w1.z + bf2f((bf16_t)v[7]) * w1.w;
      }
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (sub == 0 && b < B) {
      acc += bias;
      pred[b] = acc;
      if (target != nullptr) {
        const float diff = acc - target[b];
        lsum += diff * diff;
        if (dy != nullptr) dy[b] = dy_scale * diff;
      }
    }
  }
  if (loss_sum != nullptr) {
    const float t = block_sum<256>(lsum, red);
    if (threadIdx.x == 0) atomicAdd(loss_sum, t);
  }
}

static int lanes_per_row(int Hd) {
  int l = 1;
  while (l < 64 && l * 8 < Hd) l <<= 1;
  return l;
}

void launch_head_fwd(const bf16_t* Hm, long ldh, int B, int Hd, const float* w, const float* b0,
                     const float* target, float* pred, float* dy, float* loss_sum, float dy_scale,
                     hipStream_t s) {
  const int lpr = lanes_per_row(Hd);
  const int rpb = 256 / lpr;
  int grid = (B + rpb - 1) / rpb;
  // one same-address loss atomic per block: cap the grid. LSTM head (B = 8192, Hd = 512,
  // kernel trace, tools/gpu.sh ksweep WELLFLOW_HEAD_GRID): 30.8 us at 2048 blocks, 18.3 at 1024, 13.4 at 512,
  // 14.0 at 256 — the atomics serialise, not the loads (WELLFLOW_HEAD_GRID overrides)
  static const int cap = std::max(1, diag_env_int("WELLFLOW_HEAD_GRID", 512));  // sweep: WF_DIAG builds only
  if (grid > cap) grid = cap;
#define HEAD_FWD(L)                                                                              \
  hipLaunchKernelGGL(head_fwd_kernel<L>, dim3(grid), dim3(256), 0, s, Hm, ldh, B, Hd, w, b0, target, \
                     pred, dy, loss_sum, dy_scale)
  switch (lpr) {
    case 1: HEAD_FWD(1); break;
    case 2: HEAD_FWD(2); break;
    case 4: HEAD_FWD(4); break;
    case 8: HEAD_FWD(8); break;
    case 16: HEAD_FWD(16); break;
    case 32: HEAD_FWD(32); break;
    default: HEAD_FWD(64); break;
  }
#undef HEAD_FWD
}

// Regression head forward + MSE + head weight gradient in ONE pass over H (the LSTM's last
// hidden state): a row group of LPR lanes (LPR * 8 == Hd: each lane holds 8 columns of the row)
// forms pred, dy = s (pred - y) and the loss, then every lane adds dy * h to its 8 columns of
// dw — the h values are still in its registers, so head_bwd_w's second read of H and its
// launch disappear. kHeadRowsU rows per group are in flight at once (independent loads).
constexpr int kHeadRowsU = 16;
template <int LPR>
__global__ __launch_bounds__(256) void head_fwd_bwd_kernel(const bf16_t* __restrict__ Hm, long ldh, int B, int Hd,
                                                           const float* __restrict__ w, const float* __restrict__ b0,
                                                           const float* __restrict__ target, float* __restrict__ pred,
                                                           float* __restrict__ dy, float* __restrict__ loss_sum,
                                                           float dy_scale, float* __restrict__ dw, float* __restrict__ db) {
  // U = 16 row groups per pass: every row of a block's 64 (at H = 512) loaded at once (with 4 the
  // 128 blocks looped 4 times, one latency round each: 14.5 us for 8 MB)
  constexpr int RPB = 256 / LPR, U = kHeadRowsU;
  __shared__ float red[4];
  __shared__ float dws[RPB][LPR * 8];
  const int sub = threadIdx.x % LPR, grp = threadIdx.x / LPR;
  const float bias = b0[0];
  float wv[8], dwp[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    wv[e] = w[sub * 8 + e];
    dwp[e] = 0.f;
  }
  float lsum = 0.f, dsum = 0.f;
  for (int rb = blockIdx.x * RPB * U; rb < B; rb += gridDim.x * RPB * U) {
    bf16x8 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = rb + u * RPB + grp;
      v[u] = b < B ? *reinterpret_cast<const bf16x8*>(Hm + (size_t)b * ldh + sub * 8) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = rb + u * RPB + grp;
      float h[8], acc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        h[e] = bf2f((bf16_t)v[u][e]);
        acc += h[e] * wv[e];
      }
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (b < B) {
        const float p = acc + bias, diff = p - target[b], g = dy_scale * diff;
#pragma unroll
        for (int e = 0; e < 8; ++e) dwp[e] += g * h[e];
        if (sub == 0) {
          pred[b] = p;
          dy[b] = g;
          lsum += diff * diff;
          dsum += g;
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) dws[grp][sub * 8 + e] = dwp[e];
  __syncthreads();
  for (int col = threadIdx.x; col < Hd; col += 256) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < RPB; ++q) t += dws[q][col];
    if (t != 0.f) atomicAdd(dw + col, t);
  }
  if (loss_sum != nullptr) {
    const float t = block_sum<256>(lsum, red);
    if (threadIdx.x == 0) atomicAdd(loss_sum, t);
  }
  if (db != nullptr) {
    const float t = block_sum<256>(dsum, red);
    if (threadIdx.x == 0) atomicAdd(db, t);
  }
}

bool launch_head_fwd_bwd(const bf16_t* Hm, long ldh, int B, int Hd, const float* w, const float* b0,
                         const float* target, float* pred, float* dy, float* loss_sum, float dy_scale, float* dw,
                         float* db, hipStream_t s) {
  const int lpr = lanes_per_row(Hd);
  if (lpr * 8 != Hd || target == nullptr || dy == nullptr || dw == nullptr) return false;
  const int rows_per_block = (256 / lpr) * kHeadRowsU;
  int grid = (B + rows_per_block - 1) / rows_per_block;
  if (grid > 128) grid = 128;  // per-column atomics per block (head_bwd_w's measured cap)
#define HEAD_FB(L)                                                                                              \
  hipLaunchKernelGGL(head_fwd_bwd_kernel<L>, dim3(grid), dim3(256), 0, s, Hm, ldh, B, Hd, w, b0, target, pred, dy, \
                     loss_sum, dy_scale, dw, db)
  switch (lpr) {
    case 1: HEAD_FB(1); break;
    case 2: HEAD_FB(2); break;
    case 4: HEAD_FB(4); break;
    case 8: HEAD_FB(8); break;
    case 16: HEAD_FB(16); break;
    case 32: HEAD_FB(32); break;
    default: HEAD_FB(64); break;
  }
#undef HEAD_FB
  return true;
}

// Column-chunk x row-group layout shared by the two head backward kernels: a thread owns
// 8 consecutive units (16-B loads/stores) of rows rg, rg + RG, ...; partial column sums
// are combined through LDS and leave the block with one atomic per column.
struct HeadBwdGeom {
  int cth;  // column threads = ceil(Hd / 8)
  int rg;   // row groups per block = 256 / cth
};

__device__ __forceinline__ void colsum_block_atomic(float (&acc)[8], int cth, int c, int r, int RG,
                                                    int Hd, float* __restrict__ out, float* lds) {
  // lds: [RG][cth*8] floats; threads beyond the RG x cth grid own no slot
  if (r < RG) {
#pragma unroll
    for (int e = 0; e < 8; ++e) lds[r * cth * 8 + c * 8 + e] = acc[e];
  }
  __syncthreads();
  for (int col = threadIdx.x; col < cth * 8; col += 256) {
    float t = 0.f;
    for (int q = 0; q < RG; ++q) t += lds[q * cth * 8 + col];
    if (col < Hd) atomicAdd(out + col, t);
  }
}

// dw[u] += sum_b dy[b] h[b][u]; db += sum_b dy[b]
__global__ __launch_bounds__(256) void head_bwd_w_kernel(const bf16_t* __restrict__ Hm, long ldh,
                                                         int B, int Hd, const float* __restrict__ dy,
                                                         float* __restrict__ dw,
                                                         float* __restrict__ db, HeadBwdGeom g) {
  __shared__ float lds[256 * 8];
  __shared__ float red[4];
  const int c = threadIdx.x % g.cth, r = threadIdx.x / g.cth;
  const bool active = r < g.rg && c * 8 < Hd;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float dsum = 0.f;
  if (active) {
    for (int b = blockIdx.x * g.rg + r; b < B; b += gridDim.x * g.rg) {
      const float gy = dy[b];
      if (c == 0) dsum += gy;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(Hm + (size_t)b * ldh + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += gy * bf2f((bf16_t)v[e]);
    }
  }
  colsum_block_atomic(acc, g.cth, c, r, g.rg, Hd, dw, lds);
  if (db != nullptr) {
    const float t = block_sum<256>(dsum, red);
    if (threadIdx.x == 0) atomicAdd(db, t);
  }
}

static HeadBwdGeom head_geom(int Hd) {
  HeadBwdGeom g;
  g.cth = (Hd + 7) / 8;
  if (g.cth > 256) g.cth = 256;  // Hd <= 2048 supported
  g.rg = 256 / g.cth;
  return g;
}

void launch_head_bwd_w(const bf16_t* Hm, long ldh, int B, int Hd, const float* dy, float* dw,
                       float* db, hipStream_t s) {
  const HeadBwdGeom g = head_geom(Hd);
  int grid = (B + g.rg - 1) / g.rg;
  // per-column atomics per block: cap the grid. LSTM head (B = 8192, Hd = 512, kernel trace,
  // tools/gpu.sh ksweep WELLFLOW_HEADW_GRID): 16.2 us at 512 blocks, 11.0 at 256, 10.3 at 128, 13.6 at 64
  // (WELLFLOW_HEADW_GRID overrides)
  static const int cap = std::max(1, diag_env_int("WELLFLOW_HEADW_GRID", 128));  // sweep: WF_DIAG builds only
  if (grid > cap) grid = cap;
  hipLaunchKernelGGL(head_bwd_w_kernel, dim3(grid), dim3(256), 0, s, Hm, ldh, B, Hd, dy, dw, db, g);
}

// dz[b][u] = dy[b] * w[u] (* [h>0]); colsum[u] += sum_b dz   (16-B vector rows)
__global__ __launch_bounds__(256) void head_bwd_x_kernel(const bf16_t* __restrict__ Hm, long ldh,
                                                         int B, int Hd, const float* __restrict__ dy,
                                                         const float* __restrict__ w, int relu_mask,
                                                         bf16_t* __restrict__ dz, long ldz,
                                                         float* __restrict__ colsum, HeadBwdGeom g) {
  __shared__ float lds[256 * 8];
  const int c = threadIdx.x % g.cth, r = threadIdx.x / g.cth;
  const bool active = r < g.rg && c * 8 < Hd;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (active) {
    float wv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) wv[e] = w[c * 8 + e];
    for (int b = blockIdx.x * g.rg + r; b < B; b += gridDim.x * g.rg) {
      const float gy = dy[b];
      bf16x8 hv;
      if (relu_mask) hv = *reinterpret_cast<const bf16x8*>(Hm + (size_t)b * ldh + c * 8);
      bf16x8 out;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = gy * wv[e];
        if (relu_mask && bf2f((bf16_t)hv[e]) <= 0.f) v = 0.f;
        const bf16_t vb = f2bf(v);
        out[e] = (short)vb;
        acc[e] += bf2f(vb);
      }
      *reinterpret_cast<bf16x8*>(dz + (size_t)b * ldz + c * 8) = out;
    }
  }
  if (colsum != nullptr) colsum_block_atomic(acc, g.cth, c, r, g.rg, Hd, colsum, lds);
}

void launch_head_bwd_x(const bf16_t* Hm, long ldh, int B, int Hd, const float* dy, const float* w,
                       int relu_mask, bf16_t* dz, long ldz, float* colsum, hipStream_t s) {
  const HeadBwdGeom g = head_geom(Hd);
  int grid = (B + g.rg - 1) / g.rg;
  if (grid > 1024) grid = 1024;  // bounds same-column atomic contention (colsum)
  hipLaunchKernelGGL(head_bwd_x_kernel, dim3(grid), dim3(256), 0, s, Hm, ldh, B, Hd, dy, w,
                     relu_mask, dz, ldz, colsum, g);
}

// ---------------------------------------------------------------- multi-output losses
// kind 0: L = sum (p-y)^2,            d = scale * 2 (p-y)
// kind 1: L = sum clip(|y-p|, 0, c),  d = scale * (-sign(y-p)) * [|y-p| <= c]   (Theano grads)
// loss_sum accumulates the raw sum (host divides); dpred (bf16) feeds the backward GEMMs;
// colsum[o] += sum_b d (bias gradient of the producing layer).
__global__ __launch_bounds__(256) void loss_kernel(int kind, const float* __restrict__ pred,
                                                   const float* __restrict__ y, int B, int O,
                                                   float clip, float scale,
                                                   float* __restrict__ loss_sum,
                                                   bf16_t* __restrict__ dpred,
                                                   float* __restrict__ dpredF,
                                                   float* __restrict__ colsum) {
  __shared__ float red[4];
  __shared__ float csum[64];
  const long total = (long)B * O;
  // column sums: the launcher makes the grid stride a multiple of O (when O <= 64), so every
  // thread stays on ONE column: a register partial, one LDS add per thread and O global adds
  // per block (a global atomic per element onto O addresses took 2.7 ms at B = 65536, O = 12)
  const bool col_fixed = colsum != nullptr && O <= 64 && ((long)gridDim.x * 256) % O == 0;
  if (col_fixed && threadIdx.x < 64) csum[threadIdx.x] = 0.f;
  if (col_fixed) __syncthreads();
  float cs = 0.f;
  float ls = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const float p = pred[i], t = y[i];
    float l, d;
    if (kind == 0) {
      const float e = p - t;
      l = e * e;
      d = 2.f * e;
    } else {
      const float e = t - p, a = fabsf(e);
      l = fminf(a, clip);
      const float sg = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f);
      d = a <= clip ? -sg : 0.f;
    }
    ls += l;
    d *= scale;
    if (dpred != nullptr) dpred[i] = f2bf(d);
    if (dpredF != nullptr) dpredF[i] = d;
    if (col_fixed)
      cs += d;
    else if (colsum != nullptr)
      atomicAdd(colsum + (i % O), d);
  }
  if (col_fixed) {
    atomicAdd(&csum[(blockIdx.x * 256L + threadIdx.x) % O], cs);
    __syncthreads();
    if (threadIdx.x < O && csum[threadIdx.x] != 0.f) atomicAdd(colsum + threadIdx.x, csum[threadIdx.x]);
  }
  const float s = block_sum<256>(ls, red);
  if (threadIdx.x == 0 && loss_sum != nullptr) atomicAdd(loss_sum, s);
}

void launch_loss(int kind, const float* pred, const float* y, int B, int O, float clip, float scale,
                 float* loss_sum, bf16_t* dpred, float* dpredF, float* colsum, hipStream_t s) {
  const long total = (long)B * O;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  if (colsum != nullptr && O <= 64) {  // grid stride a multiple of O (loss_kernel column sums)
    int g = O, r = 256;
    while (r != 0) {
      const int tmp = g % r;
      g = r;
      r = tmp;
    }
    const int mult = O / g;  // blocks must be a multiple of O / gcd(256, O)
    blocks = (blocks + mult - 1) / mult * mult;
  }
  hipLaunchKernelGGL(loss_kernel, dim3(blocks), dim3(256), 0, s, kind, pred, y, B, O, clip, scale,
                     loss_sum, dpred, dpredF, colsum);
}

// ---------------------------------------------------------------- optimizers
// Adam (PyTorch semantics, decoupled weight decay when wd != 0 — AdamW form).
// bc1 = 1 - b1^t, bc2 = 1 - b2^t are computed on the host per step.
__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float lr, float b1,
                                         float b2, float eps, float wd, float bc1, float bc2) {
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  const float mh = m / bc1, vh = v / bc2;
  p -= lr * (mh / (sqrtf(vh) + eps) + wd * p);
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n,
                                                   float lr, float b1, float b2, float eps, float wd,
                                                   float bc1, float bc2, float gscale) {
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adam_one(pp.x, gg.x * gscale, mm.x, vv.x, lr, b1, b2, eps, wd, bc1, bc2);
    adam_one(pp.y, gg.y * gscale, mm.y, vv.y, lr, b1, b2, eps, wd, bc1, bc2);
    adam_one(pp.z, gg.z * gscale, mm.z, vv.z, lr, b1, b2, eps, wd, bc1, bc2);
    adam_one(pp.w, gg.w * gscale, mm.w, vv.w, lr, b1, b2, eps, wd, bc1, bc2);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride)
    adam_one(p[i], g[i] * gscale, m[i], v[i], lr, b1, b2, eps, wd, bc1, bc2);
}

static int ew_blocks(long n) {
  long b = (n / 4 + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

void launch_adam(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2,
                 float eps, float wd, float bc1, float bc2, float gscale, hipStream_t s) {
  hipLaunchKernelGGL(adam_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2,
                     eps, wd, bc1, bc2, gscale);
}

// Graph-capturable Adam: the step counter lives on the device, so a captured hipGraph
// replays with correct bias corrections. Every workgroup reads t = step[0] + 1 at entry; the
// LAST workgroup to finish (ticket in step[1]) stores it back, so no second launch is needed
// and no workgroup can see the new value early. Optional fusions: the bf16 shadow copy of
// the updated master weights (shadow != nullptr; replaces a cast launch) and zeroing the
// gradient bucket after it is consumed (zero_g; replaces the next step's fill launch).
__global__ __launch_bounds__(256) void adam_dev_kernel(float* __restrict__ p, float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       long n, float* __restrict__ step, float lr,
                                                       float b1, float b2, float eps, float wd,
                                                       float gscale, bf16_t* __restrict__ shadow, int zero_g,
                                                       bf16_t* __restrict__ tdst, long t_off, int t_rows, int t_cols) {
  const float t = step[0] + 1.f;
  const float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adam_one(pp.x, gg.x * gscale, mm.x, vv.x, lr, b1, b2, eps, wd, bc1, bc2);
    adam_one(pp.y, gg.y * gscale, mm.y, vv.y, lr, b1, b2, eps, wd, bc1, bc2);
    adam_one(pp.z, gg.z * gscale, mm.z, vv.z, lr, b1, b2, eps, wd, bc1, bc2);
    adam_one(pp.w, gg.w * gscale, mm.w, vv.w, lr, b1, b2, eps, wd, bc1, bc2);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (zero_g) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (shadow != nullptr) {
      const unsigned lo = (unsigned)f2bf(pp.x) | ((unsigned)f2bf(pp.y) << 16);
      const unsigned hi = (unsigned)f2bf(pp.z) | ((unsigned)f2bf(pp.w) << 16);
      reinterpret_cast<uint2*>(shadow)[i] = make_uint2(lo, hi);
    }
    if (tdst != nullptr) {  // transposed copy of one block (rows x cols at element t_off)
      const long e0 = 4 * i - t_off;
      if (e0 + 3 >= 0 && e0 < (long)t_rows * t_cols) {
        const float pv[4] = {pp.x, pp.y, pp.z, pp.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const long e = e0 + q;
          if (e >= 0 && e < (long)t_rows * t_cols) tdst[(e % t_cols) * t_rows + e / t_cols] = f2bf(pv[q]);
        }
      }
    }
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    adam_one(p[i], g[i] * gscale, m[i], v[i], lr, b1, b2, eps, wd, bc1, bc2);
    if (zero_g) g[i] = 0.f;
    if (shadow != nullptr) shadow[i] = f2bf(p[i]);
    const long e = i - t_off;
    if (tdst != nullptr && e >= 0 && e < (long)t_rows * t_cols) tdst[(e % t_cols) * t_rows + e / t_cols] = f2bf(p[i]);
  }
  __syncthreads();  // every thread of this workgroup has read step[0]
  if (threadIdx.x == 0) {
    unsigned* ticket = reinterpret_cast<unsigned*>(step + 1);
    if (atomicAdd(ticket, 1u) == gridDim.x - 1) {  // all other workgroups are past their read
      step[0] = t;
      *ticket = 0u;
    }
  }
}

// Adam (as adam_dev_kernel) over the LSTM's flat parameters [W G x KA | w_out | b_out] AND, in
// the same pass, the bf16 compute copies lstm_pack_weights_kernel (lstm.hip) would write next:
// Wp (gate_col row order, rows pre-scaled for the exp2-form activations) and WhhT ([H][G], the
// backward's). One launch per update instead of two (round 5; FlatAdam writeback).
__global__ __launch_bounds__(256) void lstm_adam_pack_kernel(float* __restrict__ p, float* __restrict__ g,
                                                             float* __restrict__ m, float* __restrict__ v, long n,
                                                             float* __restrict__ step, float lr, float b1, float b2,
                                                             float eps, float wd, float gscale, int zero_g, int KX, int H,
                                                             bf16_t* __restrict__ Wp, bf16_t* __restrict__ WhhT) {
  const float t = step[0] + 1.f;
  const float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
  const int KA = KX + H, G = 4 * H;
  // the W block in 32 x 32 tiles (KX, H multiples of 32, host-checked): thread = 4 consecutive
  // columns of one row, so the Adam streams and the Wp rows stay float4 / 8-B coalesced, and the
  // W_hh^T image goes out through an LDS transpose as 64-B runs of 32 rows (written straight from
  // the row-major loop it was 2-B stores 4 KiB apart: ~3x the kernel's streaming time)
  __shared__ bf16_t tt[32][36];  // [k][r]
  const int tilesK = KA / 32, ntiles = (G / 32) * tilesK;
  const int rr = threadIdx.x >> 3, kk = (threadIdx.x & 7) * 4;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int r0 = (tile / tilesK) * 32, k0 = (tile % tilesK) * 32;
    const int r = r0 + rr, k = k0 + kk;
    const long i = ((long)r * KA + k) >> 2;
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adam_one(pp.x, gg.x * gscale, mm.x, vv.x, lr, b1, b2, eps, wd, bc1, bc2);
    adam_one(pp.y, gg.y * gscale, mm.y, vv.y, lr, b1, b2, eps, wd, bc1, bc2);
    adam_one(pp.z, gg.z * gscale, mm.z, vv.z, lr, b1, b2, eps, wd, bc1, bc2);
    adam_one(pp.w, gg.w * gscale, mm.w, vv.w, lr, b1, b2, eps, wd, bc1, bc2);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (zero_g) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float sc = (r & 3) == 2 ? kLstmTanhScale : kLstmSigScale;
    const unsigned lo = (unsigned)f2bf(pp.x * sc) | ((unsigned)f2bf(pp.y * sc) << 16);
    const unsigned hi = (unsigned)f2bf(pp.z * sc) | ((unsigned)f2bf(pp.w * sc) << 16);
    *reinterpret_cast<uint2*>(Wp + (size_t)gate_col(r & 3, r >> 2) * KA + k) = make_uint2(lo, hi);
    if (k0 >= KX) {  // block-uniform: the tile lies wholly in the h columns
      tt[kk][rr] = f2bf(pp.x);
      tt[kk + 1][rr] = f2bf(pp.y);
      tt[kk + 2][rr] = f2bf(pp.z);
      tt[kk + 3][rr] = f2bf(pp.w);
      __syncthreads();
      const int kt = threadIdx.x >> 3, rc = (threadIdx.x & 7) * 4;
      const unsigned w0 = (unsigned)tt[kt][rc] | ((unsigned)tt[kt][rc + 1] << 16);
      const unsigned w1 = (unsigned)tt[kt][rc + 2] | ((unsigned)tt[kt][rc + 3] << 16);
      *reinterpret_cast<uint2*>(WhhT + (size_t)(k0 - KX + kt) * G + r0 + rc) = make_uint2(w0, w1);
      __syncthreads();
    }
  }
  // the head (w_out, b_out) past the W block
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)G * KA + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    adam_one(p[i], g[i] * gscale, m[i], v[i], lr, b1, b2, eps, wd, bc1, bc2);
    if (zero_g) g[i] = 0.f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* ticket = reinterpret_cast<unsigned*>(step + 1);
    if (atomicAdd(ticket, 1u) == gridDim.x - 1) {
      step[0] = t;
      *ticket = 0u;
    }
  }
}

void launch_lstm_adam_pack(float* p, float* g, float* m, float* v, long n, float* step, float lr, float b1, float b2,
                           float eps, float wd, float gscale, int zero_g, int KX, int H, bf16_t* Wp, bf16_t* WhhT,
                           hipStream_t s) {
  static const int cap = std::max(1, diag_env_int("WELLFLOW_ADAM_GRID", 256));
  int blocks = ew_blocks(n);
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(lstm_adam_pack_kernel, dim3(blocks), dim3(256), 0, s, p, g, m, v, n, step, lr, b1, b2, eps, wd,
                     gscale, zero_g, KX, H, Wp, WhhT);
}

void launch_adam_dev(float* p, float* g, float* m, float* v, long n, float* step, float lr,
                     float b1, float b2, float eps, float wd, float gscale, bf16_t* shadow, int zero_g,
                     hipStream_t s, bf16_t* tdst, long t_off, int t_rows, int t_cols) {
  // every workgroup draws a ticket from ONE counter (step[1]) and same-address atomics serialise:
  // at most WELLFLOW_ADAM_GRID (default 256) workgroups, grid-stride over the rest
  static const int cap = std::max(1, diag_env_int("WELLFLOW_ADAM_GRID", 256));  // sweep: WF_DIAG builds only
  int blocks = ew_blocks(n);
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(adam_dev_kernel, dim3(blocks), dim3(256), 0, s, p, g, m, v, n, step, lr,
                     b1, b2, eps, wd, gscale, shadow, zero_g, tdst, t_off, t_rows, t_cols);
}

// Keras-0.x SGD: v = mu v - lr_t g; p += mu v - lr_t g (Nesterov) or p += v.
// lr_t = lr / (1 + decay * iterations) is computed on the host.
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ vel, long n, float lr,
                                                  float momentum, int nesterov, float gscale) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gi = g[i] * gscale;
    const float v = momentum * vel[i] - lr * gi;
    vel[i] = v;
    p[i] += nesterov ? (momentum * v - lr * gi) : v;
  }
}

void launch_sgd(float* p, const float* g, float* vel, long n, float lr, float momentum,
                int nesterov, float gscale, hipStream_t s) {
  long b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(sgd_kernel, dim3((int)b), dim3(256), 0, s, p, g, vel, n, lr, momentum,
                     nesterov, gscale);
}

// Graph-capturable Keras-0.x SGD: the iteration counter lives on the device (step[0];
// step[1] is the completion ticket, as in adam_dev_kernel), so lr_t = lr / (1 + decay * it)
// advances on every hipGraph replay instead of being baked in at capture time.
__global__ __launch_bounds__(256) void sgd_dev_kernel(float* __restrict__ p, float* __restrict__ g,
                                                      float* __restrict__ vel, long n, float* __restrict__ step,
                                                      float lr, float decay, float momentum, int nesterov,
                                                      float gscale, int zero_g) {
  const float it = step[0];
  const float lr_t = lr / (1.f + decay * it);
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gi = g[i] * gscale;
    const float v = momentum * vel[i] - lr_t * gi;
    vel[i] = v;
    p[i] += nesterov ? (momentum * v - lr_t * gi) : v;
    if (zero_g) g[i] = 0.f;
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

void launch_sgd_dev(float* p, float* g, float* vel, long n, float* step, float lr, float decay, float momentum,
                    int nesterov, float gscale, int zero_g, hipStream_t s) {
  long b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(sgd_dev_kernel, dim3((int)b), dim3(256), 0, s, p, g, vel, n, step, lr, decay, momentum,
                     nesterov, gscale, zero_g);
}

// ---------------------------------------------------------------- casts
__global__ void cast_bf16_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = f2bf(src[i]);
}

void launch_cast_bf16(const float* src, bf16_t* dst, long n, hipStream_t s) {
  long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((int)b), dim3(256), 0, s, src, dst, n);
}

// ---------------------------------------------------------------- row gather
// dst[r] = src[clamp(idx[r])] for rows of row_bytes (a multiple of 4): the epoch's shuffle
// materialised once (train/trainer.py Trainer._permuted). Each thread moves VEC bytes; with
// 16-B pieces a 32-B feature row is 2 lanes and consecutive lanes cover consecutive dst rows,
// so the writes coalesce and each gathered row is one 32-B sector read (torch's index_select
// spent ~530 us on the 2.4M x 32-B MLP table, this moves it at the sector rate).
template <int VEC>
__global__ void gather_rows_kernel(const char* __restrict__ src, const long long* __restrict__ idx,
                                   char* __restrict__ dst, long m, int row_bytes, long nsrc) {
  typedef unsigned u32v __attribute__((ext_vector_type(VEC / 4)));
  const int per = row_bytes / VEC;
  const long total = m * per;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += stride) {
    const long r = i / per;
    const int c = (int)(i - r * per);
    long long sr = idx[r];
    sr = sr < 0 ? 0 : (sr >= nsrc ? nsrc - 1 : sr);
    *reinterpret_cast<u32v*>(dst + r * row_bytes + (long)c * VEC) =
        *reinterpret_cast<const u32v*>(src + sr * row_bytes + (long)c * VEC);
  }
}

void launch_gather_rows(const void* src, const long long* idx, void* dst, long m, int row_bytes, long nsrc,
                        hipStream_t s) {
  const int vec = (row_bytes % 16 == 0 && ((uintptr_t)src | (uintptr_t)dst) % 16 == 0) ? 16 : 4;
  const long total = m * (row_bytes / vec);
  long b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  if (vec == 16)
    hipLaunchKernelGGL(gather_rows_kernel<16>, dim3((int)b), dim3(256), 0, s, (const char*)src, idx, (char*)dst, m,
                       row_bytes, nsrc);
  else
    hipLaunchKernelGGL(gather_rows_kernel<4>, dim3((int)b), dim3(256), 0, s, (const char*)src, idx, (char*)dst, m,
                       row_bytes, nsrc);
}

// dst[c][r] = bf16(src[r*lds + c]) for r < rows, c < cols; 32x32 tiles through LDS.
__global__ void transpose_cast_kernel(const float* __restrict__ src, long lds, int rows, int cols,
                                      bf16_t* __restrict__ dst, long ldd) {
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    tile[k][tx] = (r < rows && c < cols) ? src[(size_t)r * lds + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (c < cols && r < rows) dst[(size_t)c * ldd + r] = f2bf(tile[tx][k]);
  }
}

void launch_transpose_cast_bf16(const float* src, long lds, int rows, int cols, bf16_t* dst,
                                long ldd, hipStream_t s) {
  dim3 grid((cols + 31) / 32, (rows + 31) / 32);
  hipLaunchKernelGGL(transpose_cast_kernel, grid, dim3(256), 0, s, src, lds, rows, cols, dst, ldd);
}

// 1-D im2col for a stride-1 valid convolution, channels-last input x[B][L][Cin]:
// col[b*Lout + t][k*Cin + c] = x[b][t+k][c] for k < ksz; column ksz*Cin is the constant 1
// (bias folded into the weight); remaining columns up to Kp are zero.
__global__ void im2col1d_kernel(const float* __restrict__ x, int B, int L, int Cin, int ksz, int Lout,
                                int Kp, bf16_t* __restrict__ col) {
  const long total = (long)B * Lout * Kp;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += stride) {
    const int kc = i % Kp;
    const long bt = i / Kp;
    const int t = bt % Lout, b = bt / Lout;
    float v = 0.f;
    if (kc < ksz * Cin) {
      const int k = kc / Cin, c = kc % Cin;
      v = x[((long)b * L + t + k) * Cin + c];
    } else if (kc == ksz * Cin) {
      v = 1.f;
    }
    col[i] = f2bf(v);
  }
}

void launch_im2col1d(const float* x, int B, int L, int Cin, int ksz, int Lout, int Kp, bf16_t* col,
                     hipStream_t s) {
  const long total = (long)B * Lout * Kp;
  long b = (total + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(im2col1d_kernel, dim3((int)b), dim3(256), 0, s, x, B, L, Cin, ksz, Lout, Kp,
                     col);
}

}  // namespace wf
