// wellflow — the MLP training step's forward AND backward in one persistent launch
// (F -> 256 -> 256 -> 1, ReLU, MSE; reference mlp.py model + train_step). SURVEY.md §2.4 K9-K11.
//
// Replaces mlp2_fwd_train_kernel + mlp2_bwd_rc8_kernel (mlp_fused.hip) for the training step:
// per 64-row chunk the X tile is staged ONCE, layer 1 runs once (the two-kernel path ran it in
// the forward and again in the backward), H2 never leaves the registers (no ReLU bitmask round
// trip through HBM) and dy never leaves the workgroup. Per chunk and wave (8 waves, wave w owns
// hidden units [32w, 32w + 32) of both layers):
//   layer 1   H1^T = relu(W1 X^T + b1)        own units -> LDS tile (bf16)        8 MFMA
//   layer 2   Z2^T = W2 H1^T                  own units, K = all of H1           64 MFMA
//   head      p = H2 w3 + b3 (partials over waves via LDS), dy = s (p - y), loss, dw3, db3
//   dZ2       = dy w3^T * [H2 > 0]            own units -> LDS tile + HBM (dW2's operand)
//   dH1^T     = W2^T dZ2^T                    own units k, K = all of dZ2        64 MFMA
//   dZ1       = dH1 * [H1 > 0]                in place over the wave's own H1 columns
//   dW1^T    += dZ1^T X                       ds_read_b64_tr_b16 fragments     2 NFT MFMA
// W1 rows and W2^T rows (dH1 A operand) stay in registers for the whole launch; layer 2's A
// operand (W2 rows) streams from L2 by buffer loads, the first K steps requested a chunk early
// (both W2 images would not fit the 256-VGPR budget of two waves per SIMD); b1 / b2 / w3 are
// read from LDS. Three workgroup barriers per chunk (H1 complete, head partials complete, dZ2
// complete — the next chunk's X / y tile is staged before the last one, which publishes it).
// Batch sums go to the spread-reduction scratch as the two kernels' did (kMlpRedCopies copies +
// the per-workgroup dW1 rows); dZ2 leaves either row-major (for mlp2_dw2) or in the fragment
// layout of the dW2 kernels below; mlp2_reduce sums everything into the gradients.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "gemm_core.h"
#include "kernels.h"
#include "mlp_tiles.h"

namespace wf {

namespace {
// FRAG: dZ2 leaves in the MFMA-fragment layout of the dW2 kernels (below) instead of [B][256]
// STAMP (WELLFLOW_MLP_STAMP=1, tools/mlp_timeline.py): lane 0 of every wave writes s_memtime at
// 13 phase boundaries of its 5th chunk into `stamps` (results unchanged)
// Loss of the one-launch steps (round 6: the reference's clipped MAE too, cnn.py:29-32): clip
// <= 0 is MSE (loss d^2, dy = dy_scale d, the caller passes dy_scale = 2 grad_scale), clip > 0 is
// mae_clip (loss min(|d|, clip), dy = dy_scale sign(d) where |d| <= clip, else 0: Theano's clip
// passes the gradient on [0, clip], d|d|/dd = sign(d) with sign(0) = 0). d = prediction - target.
__device__ __forceinline__ float step_dloss(float d, float clip) {
  if (clip <= 0.f) return d;
  return fabsf(d) <= clip ? (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) : 0.f;
}
__device__ __forceinline__ float step_loss(float d, float clip) { return clip <= 0.f ? d * d : fminf(fabsf(d), clip); }

template <int NFT, bool FRAG, bool STAMP = false>  // NFT: 16-feature tiles of dW1: 1 (Fp <= 16) or 2 (Fp <= 32)
__global__ __launch_bounds__(512, 1) void mlp2_step_kernel(
    const bf16_t* __restrict__ X, int Fp, const bf16_t* __restrict__ W1, const float* __restrict__ b1,
    const bf16_t* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ w3,
    const float* __restrict__ b3, const float* __restrict__ y, float dy_scale, float clip, int B,
    const long long* __restrict__ rows, long nrows, bf16_t* __restrict__ dZ2, float* __restrict__ pred,
    float* __restrict__ red, int prio, unsigned long long* __restrict__ stamps = nullptr) {
  constexpr int MT = 2, NW = 8, XB = MF_ROWS * MF_XROW;
  __shared__ __attribute__((aligned(16))) char xs[2 * XB];              // X tiles (double-buffered)
  __shared__ __attribute__((aligned(16))) char h1s[MF_ROWS * MF_H * 2];  // H1 -> dZ1 (own columns)
  __shared__ __attribute__((aligned(16))) char zs[MF_ROWS * MF_H * 2];   // dZ2
  __shared__ __attribute__((aligned(16))) float hred[MF_ROWS][NW];       // head partials
  __shared__ __attribute__((aligned(16))) float cst[3][MF_H];            // b1, b2, w3
  __shared__ float ys[2][MF_ROWS];
  __shared__ float lred[NW];
  // lane-private running sums of dw3, db1, db2 (float4 slot [wave][sum][m][lane] = r 0..3):
  // 24 VGPRs cheaper in LDS than in the register file. Plain read-add-write of the lane's own
  // 16 B (ds_read_b128 / ds_write_b128, conflict-free): LDS float atomics (ds_add_f32) made
  // the LDS the bottleneck of the whole kernel (PMC: LDS busy 70 %, 30 cycles per LDS op)
  __shared__ __attribute__((aligned(16))) float4 part[NW][3][2][64];

  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = tid >> 6;
  const int u0 = wid * 16 * MT;
  const int tq = l15 >> 2, tp = lane & 3;  // ds_read_b64_tr_b16 lane coordinates
  for (int i = tid; i < 3 * MF_H; i += 64 * NW) cst[i / MF_H][i % MF_H] = (i < MF_H ? b1 : i < 2 * MF_H ? b2 : w3)[i % MF_H];

  bf16x8 w1f[MT], wt[MT][8];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int u = u0 + 16 * m + l15;
    w1f[m] = 8 * g + 8 <= Fp ? *reinterpret_cast<const bf16x8*>(W1 + (size_t)u * Fp + 8 * g)
                             : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int j = 0; j < 8; ++j) wt[m][kt][j] = (short)W2[(size_t)(32 * kt + 8 * g + j) * MF_H + u];
  }
  // layer 2's A operand (W2 rows of the own units) is streamed from L2 per K step, WD steps
  // ahead: holding it too (64 VGPRs) would not fit beside W2^T in the 256-VGPR budget of two
  // waves per SIMD
  constexpr int WD = 3;
  const int w2lane = (u0 + l15) * MF_H + 8 * g;  // element offset of the lane's m = 0 fragment
  // a zero laundered per chunk (below) keeps the loads inside the chunk loop (hoisted, they
  // would pin 64 VGPRs); laundering the pointer itself would lose its global address space
  // (flat loads: counted in lgkmcnt too, so every LDS wait would wait for them)
  // Buffer loads: the per-fragment offset is an immediate / SGPR, no 64-bit address VALU.
  int w2z = 0;
  const __amdgpu_buffer_rsrc_t w2rs = __builtin_amdgcn_make_buffer_rsrc((void*)W2, 0, 0x7FFFFFFF, 0x00020000);
  auto w2frag = [&](int m, int kt) {
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    return __builtin_bit_cast(bf16x8, (u32x4_t)__builtin_amdgcn_raw_buffer_load_b128(
                                          w2rs, 2 * (w2z + w2lane), 2 * (16 * MF_H * m + 32 * kt), 0));
  };
  // the first WD K steps of layer 2, requested one chunk early (right after the previous
  // chunk's dH1 MFMAs): they land during dZ1 / dW1, the staging barrier and layer 1
  bf16x8 w2r[WD][MT];
  auto w2first = [&]() {
    w2z = 0;
    asm volatile("" : "+s"(w2z));
#pragma unroll
    for (int k = 0; k < WD; ++k)
#pragma unroll
      for (int m = 0; m < MT; ++m) w2r[k][m] = w2frag(m, k);
  };
  f32x4 dw1a[MT][NFT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int f = 0; f < NFT; ++f) dw1a[m][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < 3 * MT; ++k) part[wid][k / MT][k % MT][lane] = make_float4(0.f, 0.f, 0.f, 0.f);
  auto acc4 = [&](int P, int m, const float (&v)[4]) {
    float4 a = part[wid][P][m][lane];
    a.x += v[0];
    a.y += v[1];
    a.z += v[2];
    a.w += v[3];
    part[wid][P][m][lane] = a;
  };
  constexpr int P_DW3 = 0, P_DB1 = 1, P_DB2 = 2;
  const float bias3 = b3[0];
  float lsum = 0.f, db3a = 0.f;

  // next chunk's inputs: threads 0..255 one 16-B X row segment each (row t >> 2, chunk t & 3),
  // threads 256..319 one target
  uint4 xv = make_uint4(0, 0, 0, 0);
  float yv = 0.f;
  auto prefetch = [&](int ch) {
    if (tid < 256) {
      const int r = tid >> 2, c = tid & 3, gr = ch * MF_ROWS + r;
      xv = (gr < B && 8 * c + 8 <= Fp) ? *reinterpret_cast<const uint4*>(X + data_row(rows, gr, nrows) * Fp + 8 * c)
                                       : make_uint4(0, 0, 0, 0);
    } else if (tid < 256 + MF_ROWS) {
      const int gr = ch * MF_ROWS + tid - 256;
      yv = gr < B ? y[data_row(rows, gr, nrows)] : 0.f;
    }
  };
  const int nchunks = (B + MF_ROWS - 1) / MF_ROWS;
  auto stage = [&](int p) {  // the prefetched chunk -> X / y buffer p
    if (tid < 256)
      *reinterpret_cast<uint4*>(xs + p * XB + xtile_off(tid >> 2, tid & 3)) = xv;
    else if (tid < 256 + MF_ROWS)
      ys[p][tid - 256] = yv;
  };
  if ((int)blockIdx.x < nchunks) prefetch(blockIdx.x);
  // first chunk staged here (its barrier also publishes cst), the second one prefetched; every
  // later chunk is staged before the previous chunk's dZ2 barrier, which publishes it (three
  // workgroup barriers per chunk; the four-barrier order measured 0.4 % slower, r4/final)
  stage(0);
  __syncthreads();
  if ((int)blockIdx.x + (int)gridDim.x < nchunks) prefetch(blockIdx.x + gridDim.x);
  w2first();
  // static priority for the second-dispatched half (waves 4-7), which otherwise loses every VALU
  // arbitration to its SIMD partner (MI355X_MICROARCH.md "two waves per SIMD", item 4)
  if (prio && __builtin_amdgcn_readfirstlane(wid) >= 4) __builtin_amdgcn_s_setprio(1);
  int par = 0;
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x, par ^= 1) {
    const int row0 = ch * MF_ROWS;
    auto stamp = [&](int k) {
      if constexpr (STAMP) {
        if (ch == (int)blockIdx.x + 4 * (int)gridDim.x && lane == 0)
          stamps[((size_t)blockIdx.x * NW + wid) * 16 + k] = __builtin_amdgcn_s_memtime();
      }
    };
    stamp(0);
    char* xt = xs + par * XB;
    stamp(1);

    // ---- layer 1 (own units): H1 -> h1s; the first W2 fragments of layer 2 in flight
    f32x4 acc[MT][4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const bf16x8 xb = *reinterpret_cast<const bf16x8*>(xt + xtile_off(16 * n + l15, g));
#pragma unroll
      for (int m = 0; m < MT; ++m)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[m], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float4 bb = *reinterpret_cast<const float4*>(&cst[0][u0 + 16 * m + 4 * g]);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const unsigned p0 = pk_bf16(fmaxf(acc[m][n][0] + bb.x, 0.f), fmaxf(acc[m][n][1] + bb.y, 0.f));
        const unsigned p1 = pk_bf16(fmaxf(acc[m][n][2] + bb.z, 0.f), fmaxf(acc[m][n][3] + bb.w, 0.f));
        *reinterpret_cast<uint2*>(h1s + tile_off(16 * n + l15, u0 + 16 * m + 4 * g)) = make_uint2(p0, p1);
      }
    }
    stamp(2);
    __syncthreads();  // B2: H1 complete
    stamp(3);

    // ---- layer 2 (own units, K = 256)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    // H1 fragments rotate through ONE set of 4 registers: fragment n of K step kt + 1 is read
    // right after the two MFMAs that consume fragment n of step kt (their operands are read at
    // issue), so each read has 6 MFMAs of cover and no extra VGPRs. The compiler otherwise
    // issued all 4 reads of a step in front of its MFMAs and waited for each (the layer ran at
    // 5.9k cycles per chunk against 2.0k for dH1, which it happened to pipeline).
    bf16x8 hb[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) hb[n] = *reinterpret_cast<const bf16x8*>(h1s + tile_off(16 * n + l15, 8 * g));
    static_for<0, 8>([&](auto kc) {
      constexpr int kt = decltype(kc)::value;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2r[kt % WD][m], hb[n], acc[m][n], 0, 0, 0);
        if constexpr (kt + 1 < 8) {
          __builtin_amdgcn_sched_barrier(0);  // keep the read here: the scheduler sinks it to its use
          hb[n] = *reinterpret_cast<const bf16x8*>(h1s + tile_off(16 * n + l15, 32 * (kt + 1) + 8 * g));
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if constexpr (kt + WD < 8) {  // refill the W2 slot just consumed
#pragma unroll
        for (int m = 0; m < MT; ++m) w2r[kt % WD][m] = w2frag(m, kt + WD);
      }
    });
    stamp(4);
    // H2 = relu(Z2 + b2) rounded to bf16 (the stored-activation numerics of the reference
    // path), kept in acc; head partials of rows 16n + l15
    float hp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float4 bb = *reinterpret_cast<const float4*>(&cst[1][u0 + 16 * m + 4 * g]);
      const float4 ww = *reinterpret_cast<const float4*>(&cst[2][u0 + 16 * m + 4 * g]);
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w}, wv[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = bf2f(f2bf(fmaxf(acc[m][n][r] + bv[r], 0.f)));
          acc[m][n][r] = v;
          hp[n] += v * wv[r];
        }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      hp[n] += __shfl_xor(hp[n], 16, 64);
      hp[n] += __shfl_xor(hp[n], 32, 64);
    }
    if (g == 0) {
#pragma unroll
      for (int n = 0; n < 4; ++n) hred[16 * n + l15][wid] = hp[n];
    }
    stamp(5);
    __syncthreads();  // B3: head partials complete
    stamp(6);

    // ---- prediction, dy, loss of rows 16n + l15 (every wave needs dy); wave 0 lane group g
    // owns row 16g + l15's outputs
    float dyn[4], pst = 0.f;
    int pgr = -1;  // the prediction this lane stores (after the next W2 request, below)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int r = 16 * n + l15, gr = row0 + r;
      const float4 pa = *reinterpret_cast<const float4*>(&hred[r][0]);
      const float4 pb = *reinterpret_cast<const float4*>(&hred[r][4]);
      const float p = ((pa.x + pa.y) + (pa.z + pa.w)) + ((pb.x + pb.y) + (pb.z + pb.w)) + bias3;
      dyn[n] = 0.f;
      if (gr < B) {
        const float diff = p - ys[par][r];
        dyn[n] = dy_scale * step_dloss(diff, clip);
        if (wid == 0 && g == n) {
          pst = p;
          pgr = gr;
          lsum += step_loss(diff, clip);
          db3a += dyn[n];
        }
      }
    }
    // ---- dZ2 = dy w3^T * [H2 > 0] (own units) -> zs; dw3, db2 partials (fp32, pre-rounding)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float4 ww = *reinterpret_cast<const float4*>(&cst[2][u0 + 16 * m + 4 * g]);
      const float wv[4] = {ww.x, ww.y, ww.z, ww.w};
      float s3[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        float t[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s3[r] += acc[m][n][r] * dyn[n];
          t[r] = acc[m][n][r] > 0.f ? dyn[n] : 0.f;
          s2[r] += t[r];
        }
        *reinterpret_cast<uint2*>(zs + tile_off(16 * n + l15, u0 + 16 * m + 4 * g)) =
            make_uint2(pk_bf16(t[0] * wv[0], t[1] * wv[1]), pk_bf16(t[2] * wv[2], t[3] * wv[3]));
      }
      acc4(P_DW3, m, s3);
      acc4(P_DB2, m, s2);
    }
    // the next chunk's X / y into the other buffer (its last readers — layer 1 and dW1 of the
    // previous chunk — are behind this chunk's B2), published by B4
    if (ch + (int)gridDim.x < nchunks) stage(par ^ 1);
    stamp(7);
    __syncthreads();  // B4: dZ2 complete, next chunk's X / y staged
    stamp(8);
    if (ch + 2 * (int)gridDim.x < nchunks) prefetch(ch + 2 * gridDim.x);

    stamp(9);
    // ---- dH1^T (own units k, K = 256 output units) = W2^T dZ2^T
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      bf16x8 zb[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) zb[n] = *reinterpret_cast<const bf16x8*>(zs + tile_off(16 * n + l15, 32 * kt + 8 * g));
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wt[m][kt], zb[n], acc[m][n], 0, 0, 0);
    }
    stamp(10);
    w2first();  // the next chunk's first layer-2 fragments
    // Global stores only AFTER that request: vmcnt counts stores too and completes in order, so
    // a store issued before a load holds every wait for that load until the store is
    // acknowledged — with the dZ2 copy-out before dH1, layer 2 of the next chunk waited on it
    // (5.9k cycles per chunk against a 2.0k MFMA floor, tools/mlp_timeline.py)
    if (pgr >= 0 && pred != nullptr) pred[pgr] = pst;
    if constexpr (FRAG) {
      // ---- dZ2 copy-out as dW2 A fragments: fragment (s, b) = 32 rows x 16 units, lane
      // (l15, g) 16 B = rows 32s + 8g .. + 7 of unit 16b + l15 (two ds_read_b64_tr_b16); wave w
      // writes fragments 4w .. 4w + 3, one coalesced 1-KiB store each (B % 64 == 0)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = 4 * wid + q, sst = f >> 4, b = f & 15;
        bf16x8 v;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bf16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(zs + tile_off(32 * sst + 8 * g + 4 * h + tq, 16 * b + 4 * tp)));
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * h + e] = t[e];
        }
        const size_t S = (size_t)(row0 >> 5) + sst;
        *reinterpret_cast<bf16x8*>(dZ2 + ((S * 16 + b) * 64 + lane) * 8) = v;
      }
    } else {
      // ---- dZ2 copy-out: 16-B row segments, thread t always chunk t & 31 (coalesced 512-B rows)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (tid >> 5) + 16 * i, c = tid & 31;
        if (row0 + r < B)
          *reinterpret_cast<uint4*>(dZ2 + (size_t)(row0 + r) * MF_H + 8 * c) =
              *reinterpret_cast<const uint4*>(zs + tile_off(r, 8 * c));
      }
    }
    // ---- dZ1 = dH1 * [H1 > 0] over the same 8 bytes of h1s; db1 partials
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float s1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int r = 16 * n + l15;
        uint2* pp = reinterpret_cast<uint2*>(h1s + tile_off(r, u0 + 16 * m + 4 * g));
        const uint2 hv = *pp;
        const bool rok = row0 + r < B;
        const int hw2[2] = {rok ? (int)hv.x : 0, rok ? (int)hv.y : 0};
        unsigned ow[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          // H1 >= 0 (relu): H1 > 0 <=> the bf16 half is > 0 as a signed 16-bit integer
          const bool on0 = (hw2[q] << 16) > 0, on1 = hw2[q] > 0xFFFF;
          const float t0 = on0 ? acc[m][n][2 * q] : 0.f, t1 = on1 ? acc[m][n][2 * q + 1] : 0.f;
          s1[2 * q] += t0;
          s1[2 * q + 1] += t1;
          ow[q] = pk_bf16(t0, t1);
        }
        *pp = make_uint2(ow[0], ow[1]);
      }
      acc4(P_DB1, m, s1);
    }
    stamp(11);
    // the dW1 fragments read other lanes' dZ1 (same wave): complete the writes first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // ---- dW1^T slice (32 units x Fp) += dZ1^T X over the chunk's rows
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MT], bfr[NFT];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 32 * kk + 8 * g + 4 * h + tq;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(h1s + tile_off(r, u0 + 16 * m + 4 * tp)));
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
    // h1s columns are rewritten by this wave's next layer 1: its dW1 reads must be complete
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    stamp(12);
  }

  // ---- batch sums -> copy blockIdx % kMlpRedCopies of the scratch; dW1 -> this workgroup's row
  float* rb = red + (blockIdx.x & (kMlpRedCopies - 1)) * kMlpRedRow;
  float* slab = red + kMlpRedSlabOff + (size_t)blockIdx.x * kMlpRedSlabRow;
  const float tl = block_sum<512>(lsum, lred);
  if (tid == 0 && tl != 0.f) atomicAdd(rb + kMlpRedLoss, tl);
  const float t3 = block_sum<512>(db3a, lred);
  if (tid == 0 && t3 != 0.f) atomicAdd(rb + kMlpRedDb3, t3);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int u = u0 + 16 * m + 4 * g + r;
      const float4 a3 = part[wid][P_DW3][m][lane], a1 = part[wid][P_DB1][m][lane], a2 = part[wid][P_DB2][m][lane];
      const float pick3[4] = {a3.x, a3.y, a3.z, a3.w}, pick1[4] = {a1.x, a1.y, a1.z, a1.w},
                  pick2[4] = {a2.x, a2.y, a2.z, a2.w};
      float v[3] = {pick3[r], pick1[r], pick2[r] * cst[2][u]};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        v[k] += __shfl_xor(v[k], 1, 64);
        v[k] += __shfl_xor(v[k], 2, 64);
        v[k] += __shfl_xor(v[k], 4, 64);
        v[k] += __shfl_xor(v[k], 8, 64);
      }
      if (l15 == 0) {
        if (v[0] != 0.f) atomicAdd(rb + kMlpRedDw3 + u, v[0]);
        if (v[1] != 0.f) atomicAdd(rb + kMlpRedDb1 + u, v[1]);
        if (v[2] != 0.f) atomicAdd(rb + kMlpRedDb2 + u, v[2]);
      }
    }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int f = 0; f < NFT; ++f) {
      const int ft = l15 + 16 * f;
      if (ft < Fp)
#pragma unroll
        for (int i = 0; i < 4; ++i) slab[(u0 + 16 * m + 4 * g + i) * Fp + ft] = dw1a[m][f][i];
    }
}

// ----------------------------------------------------------------------------------------
// 128-row passes (round-4 VERDICT item 3): the same step as mlp2_step_kernel over TWO 64-row
// chunks at a time, with BOTH layer-2 weight images streamed from L2 — W2 rows for layer 2 and
// W2^T rows (a transposed bf16 copy the optimizer / sync_weights writes) for dH1 — so every
// streamed fragment feeds 8 row tiles instead of 4: per row, L2 bytes halve for layer 2 and the
// 64 VGPRs of the resident W2^T image pay for the doubled accumulators (acc[2][8]). The two
// GEMMs run one continuous 16-step fragment stream per pass (8 W2 K-steps, then 8 W2^T K-steps,
// WD = 4 slots ahead; 16 % WD == 0 keeps every slot index static). Batch sums live in registers
// (the 48-KiB LDS sum block of the 64-row kernel does not fit beside the 128-row tiles).
// LDS: X (double-buffered, 64-B rows, Fp <= 32) 16 KiB + H1 64 KiB + dZ2 64 KiB + head 4 KiB.
// Fp <= 64 (NFT = 4, round 6): 128-B X rows, two layer-1 K steps and ONE X buffer (two would
// not fit beside H1 and dZ2), staged at the top of each pass between two barriers.
// Rows past B are masked (dy = 0, no stores); FRAG fragments of rows >= B are not written.
__device__ __forceinline__ int x4_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }
// 128-B rows: 16-B chunk c of row r at slot c ^ ((r >> 1) & 7), so the layer-1 fragment reads
// (rows 16n + l15, chunks g / g + 4) hit 16 distinct 16-B slots in every ds_read_b128 lane group
template <int XW>
__device__ __forceinline__ int x_off(int row, int chunk) {
  if constexpr (XW == 64)
    return x4_off(row, chunk);
  else
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// Packed-bf16 epilogue helpers of the 128-row kernel (round 5: its passes were VALU-bound —
// 1.5k VALU vs 280 MFMA per wave and pass, 20 % MFMA busy, profiles/r5/pmc_mlp):
//   relu_pk: ReLU of a packed pair, one v_pk_max_i16 (a negative bf16 is a negative int16, and
//            relu(round(x)) == round(relu(x)) bit for bit);
//   mask_pk: "d where h != 0" per 16-bit half, v_pk_min_u16 + v_pk_mul_lo_u16 (h is a ReLU
//            output >= 0, so min(h, 1) is the 0/1 mask); asm because the compiler rewrites the
//            pair into two compares, two selects and a merge.
typedef short s16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned relu_pk(unsigned p) {
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, p), (s16x2_t){0, 0}));
}
__device__ __forceinline__ unsigned mask_pk(unsigned d, unsigned h) {
  unsigned o;
  asm("v_pk_min_u16 %0, %1, %3\n\tv_pk_mul_lo_u16 %0, %2, %0" : "=&v"(o) : "v"(h), "v"(d), "s"(0x00010001u));
  return o;
}
__device__ __forceinline__ f32x2_t bf_lo_hi(unsigned q) {  // packed bf16 pair -> two floats
  return f32x2_t{__uint_as_float(q << 16), __uint_as_float(q & 0xFFFF0000u)};
}

// STAMP (WELLFLOW_MLP_STAMP=1 in a WF_DIAG build, tools/mlp_timeline.py --k128): lane 0 of every
// wave writes s_memtime at 13 phase boundaries of its 3rd pass into `stamps` (results unchanged)
template <int NFT, bool STAMP = false>  // NFT: 16-feature tiles of dW1: 1, 2 or 4 (Fp <= 16 / 32 / 64)
__global__ __launch_bounds__(512, 1) void mlp2_step128_kernel(
    const bf16_t* __restrict__ X, int Fp, const bf16_t* __restrict__ W1, const float* __restrict__ b1,
    const bf16_t* __restrict__ W2, const bf16_t* __restrict__ W2T, const float* __restrict__ b2,
    const float* __restrict__ w3, const float* __restrict__ b3, const float* __restrict__ y, float dy_scale, float clip,
    int B,
    const long long* __restrict__ rows, long nrows, bf16_t* __restrict__ dZ2, float* __restrict__ pred,
    float* __restrict__ red, int prio, unsigned long long* __restrict__ stamps = nullptr) {
  constexpr int MT = 2, NR = 8, NW = 8, R = 128, WD = 4;
  constexpr int KT1 = NFT > 2 ? 2 : 1;  // layer-1 K steps of 32 features
  constexpr bool SB = KT1 == 2;         // one X buffer, staged at the pass top
  constexpr int XW = 64 * KT1, CPR = XW / 16, XB = R * XW, NP = R * CPR / 512;  // row bytes, chunks / row, pieces / thread
  static_assert(16 % WD == 0, "stream slots must repeat every pass");
  __shared__ __attribute__((aligned(16))) char xs[(SB ? 1 : 2) * XB];  // X tiles (double-buffered for KT1 = 1)
  __shared__ __attribute__((aligned(16))) char h1s[R * MF_H * 2];   // H1 -> dZ1 (own columns)
  __shared__ __attribute__((aligned(16))) char zs[R * MF_H * 2];    // dZ2
  __shared__ __attribute__((aligned(16))) float hred[R][NW + 4];    // head partials (48-B rows: conflict-free float4 reads)
  __shared__ __attribute__((aligned(16))) float cst[3][MF_H];       // b1, b2, w3
  __shared__ float ys[2][R];
  __shared__ float lred[NW];

  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = tid >> 6;
  const int u0 = wid * 16 * MT;
  const int tq = l15 >> 2, tp = lane & 3;  // ds_read_b64_tr_b16 lane coordinates
  for (int i = tid; i < 3 * MF_H; i += 64 * NW) cst[i / MF_H][i % MF_H] = (i < MF_H ? b1 : i < 2 * MF_H ? b2 : w3)[i % MF_H];

  // W1 fragments: resident for KT1 = 1; KT1 = 2 re-reads them (L2) at every pass top so their
  // 16 VGPRs are free through the stream loops (resident, the kernel spilled 73 VGPRs)
  bf16x8 w1f[MT][KT1];
  auto load_w1 = [&](int z) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int k = 0; k < KT1; ++k) {
        const int u = u0 + 16 * m + l15, f = 32 * k + 8 * g;
        w1f[m][k] = f + 8 <= Fp ? *reinterpret_cast<const bf16x8*>(W1 + (size_t)(u * Fp + f + z))
                                : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
  };
  if constexpr (!SB) load_w1(0);
  // the fragment stream: step s < 8 = W2 K-step s (layer 2), 8 <= s < 16 = W2^T K-step s - 8
  // (dH1); lane fragment (m, kt) = 16 B at row u0 + 16m + l15, columns 32kt + 8g (both images
  // are [256][256] row-major, so one offset formula serves both resources)
  int w2z = 0;  // laundered zero: keeps the loads inside the pass loop (hoisted they pin VGPRs)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)W2, 0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsT = __builtin_amdgcn_make_buffer_rsrc((void*)W2T, 0, 0x7FFFFFFF, 0x00020000);
  const int wlane = (u0 + l15) * MF_H + 8 * g;
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  auto wfrag = [&](int s, int m) {
    const int kt = s & 7;
    return __builtin_bit_cast(bf16x8, (u32x4_t)__builtin_amdgcn_raw_buffer_load_b128(
                                          s < 8 ? rsA : rsT, 2 * (w2z + wlane), 2 * (16 * MF_H * m + 32 * kt), 0));
  };
  bf16x8 wr[WD][MT];
  auto wfirst = [&]() {  // stream steps 0 .. WD - 1 (the next pass's first layer-2 fragments)
    w2z = 0;
    asm volatile("" : "+s"(w2z));
#pragma unroll
    for (int s = 0; s < WD; ++s)
#pragma unroll
      for (int m = 0; m < MT; ++m) wr[s][m] = wfrag(s, m);
  };
  f32x4 dw1a[MT][NFT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int f = 0; f < NFT; ++f) dw1a[m][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  // batch sums: dw3 partials as fp32 pairs (the lane's row, units 4g + {0, 1} and 4g + {2, 3});
  // db1 and db2 as MFMA accumulators against an all-ones B operand — the column sums of the
  // bf16 dZ1 / dZ2 fragments the dW1 and copy-out phases already hold (A layout: M = units,
  // K = rows), 16 MFMAs per pass instead of ~250 VALU of masked fp32 adds
  f32x2_t s3[MT][2];
  f32x4 db1a[MT], db2a[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    s3[m][0] = s3[m][1] = f32x2_t{0.f, 0.f};
    db1a[m] = db2a[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8 ones = __builtin_bit_cast(bf16x8, (u32x4_t{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u}));
  const float bias3 = b3[0];
  float lsum = 0.f, db3a = 0.f;

  // next pass's inputs: thread t NP 16-B X segments (piece t + 512k: row (t + 512k) / CPR, chunk
  // t % CPR), the chunk-0 threads the target of their row. Row-indexed batches (rows != nullptr, nrows < 2^31): a pass's dataset row
  // ids are loaded one pass before its gathers — loaded right before them, the dependent wait
  // after B4 also drained every W2^T stream fragment in flight
  uint4 xv[NP];
  float yv[NP];
  int ixn[NP];  // clamped row ids (of the piece rows) of the pass the next prefetch() gathers
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    xv[k] = make_uint4(0, 0, 0, 0);
    yv[k] = 0.f;
    ixn[k] = 0;
  }
  auto fetch_ids = [&](int ps, int tid) {
    if (rows != nullptr) {
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const int gr = ps * R + (tid + 512 * k) / CPR;
        const long long r = gr < B ? rows[gr] : 0;
        ixn[k] = (int)(r < 0 ? 0 : (r >= nrows ? nrows - 1 : r));
      }
    }
  };
  auto prefetch = [&](int ps, int tid) {
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int r = (tid + 512 * k) / CPR, c = tid % CPR, gr = ps * R + r;
      const size_t xr = rows != nullptr ? (size_t)ixn[k] : (size_t)gr;
      xv[k] = (gr < B && 8 * c + 8 <= Fp) ? *reinterpret_cast<const uint4*>(X + xr * Fp + 8 * c) : make_uint4(0, 0, 0, 0);
      if (c == 0) yv[k] = gr < B ? y[xr] : 0.f;
    }
  };
  const int npass = (B + R - 1) / R;
  auto stage = [&](int p, int tid) {
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int r = (tid + 512 * k) / CPR, c = tid % CPR;
      *reinterpret_cast<uint4*>(xs + p * XB + x_off<XW>(r, c)) = xv[k];
      if (c == 0) ys[p][r] = yv[k];
    }
  };
  const int G = gridDim.x;
  if ((int)blockIdx.x < npass) {
    fetch_ids(blockIdx.x, tid);
    prefetch(blockIdx.x, tid);
  }
  stage(0, tid);
  __syncthreads();
  if constexpr (SB) {  // pass b + G is prefetched after B4 of pass b
    if ((int)blockIdx.x + G < npass) fetch_ids(blockIdx.x + G, tid);
  } else {
    if ((int)blockIdx.x + G < npass) {
      fetch_ids(blockIdx.x + G, tid);
      prefetch(blockIdx.x + G, tid);
    }
    if ((int)blockIdx.x + 2 * G < npass) fetch_ids(blockIdx.x + 2 * G, tid);
  }
  wfirst();
  if (prio && __builtin_amdgcn_readfirstlane(wid) >= 4) __builtin_amdgcn_s_setprio(1);
  int par = 0;
  for (int ps = blockIdx.x; ps < npass; ps += G, par ^= 1) {
    const int row0 = ps * R;
    auto stamp = [&](int k) {
      if constexpr (STAMP) {
        if (ps == (int)blockIdx.x + 2 * G && lane == 0)
          stamps[((size_t)blockIdx.x * NW + wid) * 16 + k] = __builtin_amdgcn_s_memtime();
      }
    };
    if constexpr (SB) {
      int w1z = 0;  // laundered zero: the loads stay in the loop (hoisted they pin 16 VGPRs)
      asm volatile("" : "+s"(w1z));
      load_w1(w1z);
      if (ps != (int)blockIdx.x) {  // every wave's dW1 reads of the previous X are done: stage
        __syncthreads();
        stage(0, tid);
        __syncthreads();
      }
    }
    const int xbuf = SB ? 0 : par;  // this pass's X / target buffer
    stamp(0);
    char* xt = xs + xbuf * XB;
    // the lane coordinates, laundered per pass: every LDS address below derives from them, and
    // as loop invariants the compiler hoisted ~40 swizzled addresses out of the pass loop and
    // spilled them (one VGPR each); recomputed here they live for one phase
    int lnv = lane, tdv = tid;
    asm volatile("" : "+v"(lnv), "+v"(tdv));
    const int l15 = lnv & 15, g = lnv >> 4, tq = l15 >> 2, tp = lnv & 3;

    // ---- layer 1 (own units, 8 row tiles): H1 = relu(W1 X^T + b1) -> h1s; b1 enters as the
    // MFMA's C operand, the ReLU on the packed bf16 pair
    f32x4 acc[MT][NR];
    {
      f32x4 bv[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const float4 bb = *reinterpret_cast<const float4*>(&cst[0][u0 + 16 * m + 4 * g]);
        bv[m] = f32x4{bb.x, bb.y, bb.z, bb.w};
      }
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        bf16x8 xb[KT1];
#pragma unroll
        for (int k = 0; k < KT1; ++k) xb[k] = *reinterpret_cast<const bf16x8*>(xt + x_off<XW>(16 * n + l15, g + 4 * k));
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[m][0], xb[0], bv[m], 0, 0, 0);
          if constexpr (KT1 == 2) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[m][1], xb[1], acc[m][n], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        const unsigned p0 = relu_pk(pk_bf16(acc[m][n][0], acc[m][n][1]));
        const unsigned p1 = relu_pk(pk_bf16(acc[m][n][2], acc[m][n][3]));
        *reinterpret_cast<uint2*>(h1s + tile_off(16 * n + l15, u0 + 16 * m + 4 * g)) = make_uint2(p0, p1);
      }
    stamp(1);
    __syncthreads();  // B2: H1 complete
    stamp(2);

    // ---- layer 2 (own units, K = 256): stream steps 0..7; the B fragments (H1) rotate through
    // one set of NR registers, fragment n of K step kt + 1 read right after its two MFMAs of kt;
    // b2 is the first K step's C operand
    f32x4 bv2[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float4 bb = *reinterpret_cast<const float4*>(&cst[1][u0 + 16 * m + 4 * g]);
      bv2[m] = f32x4{bb.x, bb.y, bb.z, bb.w};
    }
    bf16x8 hb[NR];
#pragma unroll
    for (int n = 0; n < NR; ++n) hb[n] = *reinterpret_cast<const bf16x8*>(h1s + tile_off(16 * n + l15, 8 * g));
    static_for<0, 8>([&](auto kc) {
      constexpr int kt = decltype(kc)::value;
#pragma unroll
      for (int n = 0; n < NR; ++n) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[kt % WD][m], hb[n], kt == 0 ? bv2[m] : acc[m][n], 0, 0, 0);
        if constexpr (kt + 1 < 8) {
          __builtin_amdgcn_sched_barrier(0);
          hb[n] = *reinterpret_cast<const bf16x8*>(h1s + tile_off(16 * n + l15, 32 * (kt + 1) + 8 * g));
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) wr[kt % WD][m] = wfrag(kt + WD, m);  // steps WD .. 7 + WD (W2^T from 8)
    });
    stamp(3);
    // H2 = relu(Z2 + b2) rounded to bf16 (packed ReLU), kept in acc as floats; head partials of
    // rows 16n + l15 as packed fp32 FMAs over unit pairs
    f32x2_t hp2[NR];
#pragma unroll
    for (int n = 0; n < NR; ++n) hp2[n] = f32x2_t{0.f, 0.f};
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float4 ww = *reinterpret_cast<const float4*>(&cst[2][u0 + 16 * m + 4 * g]);
      const f32x2_t w01{ww.x, ww.y}, w23{ww.z, ww.w};
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        const f32x2_t v01 = bf_lo_hi(relu_pk(pk_bf16(acc[m][n][0], acc[m][n][1])));
        const f32x2_t v23 = bf_lo_hi(relu_pk(pk_bf16(acc[m][n][2], acc[m][n][3])));
        acc[m][n] = f32x4{v01.x, v01.y, v23.x, v23.y};
        hp2[n] = __builtin_elementwise_fma(v01, w01, hp2[n]);
        hp2[n] = __builtin_elementwise_fma(v23, w23, hp2[n]);
      }
    }
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      // sum over the 4 lane groups with two VALU lane swaps (v_permlane32/16_swap; the shuffles
      // went through the LDS pipe): lanes 0-15 end with the row's partial over all 32 units
      float hp = hp2[n].x + hp2[n].y;
      const unsigned hu = __float_as_uint(hp);
      hp += __uint_as_float(__builtin_amdgcn_permlane32_swap(hu, hu, false, false)[1]);  // + lane l + 32
      const unsigned tu = __float_as_uint(hp);
      hp += __uint_as_float(__builtin_amdgcn_permlane16_swap(tu, tu, false, false)[1]);  // + lane l + 16
      if (g == 0) hred[16 * n + l15][wid] = hp;
    }
    stamp(4);
    __syncthreads();  // B3: head partials complete
    stamp(5);

    // ---- prediction, dy of rows 16n + l15 (every wave needs dy), branch-free; wave 0 lane group
    // g owns rows 16n + l15 for n = g and g + 4 (their loss, db3 and prediction store): selected
    // on the way, accounted after the loop (per-row branches here cost ~1.8k cycles per pass)
    float dyn[NR], pq[2] = {0.f, 0.f}, dq[2] = {0.f, 0.f};
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      const int r = 16 * n + l15;
      const float4 pa = *reinterpret_cast<const float4*>(&hred[r][0]);
      const float4 pb = *reinterpret_cast<const float4*>(&hred[r][4]);
      const float p = ((pa.x + pa.y) + (pa.z + pa.w)) + ((pb.x + pb.y) + (pb.z + pb.w)) + bias3;
      const float diff = p - ys[xbuf][r];
      dyn[n] = row0 + r < B ? dy_scale * step_dloss(diff, clip) : 0.f;
      const bool own = (n & 3) == g;
      pq[n >> 2] = own ? p : pq[n >> 2];
      dq[n >> 2] = own ? diff : dq[n >> 2];
      if (n & 1) __builtin_amdgcn_sched_barrier(0);  // <= 4 head float4 reads in flight (VGPRs)
    }
    float pst[2] = {0.f, 0.f};
    int pgr[2] = {-1, -1};
    if (wid == 0) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int gr = row0 + 16 * (g + 4 * q) + l15;
        const bool ok = gr < B;
        pst[q] = pq[q];
        pgr[q] = ok ? gr : -1;
        lsum += ok ? step_loss(dq[q], clip) : 0.f;
        db3a += ok ? dy_scale * step_dloss(dq[q], clip) : 0.f;
      }
    }
    stamp(6);
    // ---- dZ2 = bf16(dy w3) where H2 > 0 (own units) -> zs; dw3 partials. The product is rounded
    // first and masked on the packed pair (the same bits as rounding the masked product)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float4 ww = *reinterpret_cast<const float4*>(&cst[2][u0 + 16 * m + 4 * g]);
      const f32x2_t w01{ww.x, ww.y}, w23{ww.z, ww.w};
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        const f32x2_t dd{dyn[n], dyn[n]};
        const f32x2_t v01{acc[m][n][0], acc[m][n][1]}, v23{acc[m][n][2], acc[m][n][3]};
        s3[m][0] = __builtin_elementwise_fma(v01, dd, s3[m][0]);
        s3[m][1] = __builtin_elementwise_fma(v23, dd, s3[m][1]);
        const f32x2_t z01 = dd * w01, z23 = dd * w23;
        const unsigned d0 = mask_pk(pk_bf16(z01.x, z01.y), pk_bf16(v01.x, v01.y));
        const unsigned d1 = mask_pk(pk_bf16(z23.x, z23.y), pk_bf16(v23.x, v23.y));
        *reinterpret_cast<uint2*>(zs + tile_off(16 * n + l15, u0 + 16 * m + 4 * g)) = make_uint2(d0, d1);
      }
    }
    // the sums materialised HERE: left to itself the compiler sank these adds to the end of the
    // pass and kept all 64 H2 values alive through dH1 — 200+ spilled VGPRs
#pragma unroll
    for (int m = 0; m < MT; ++m) asm volatile("" : "+v"(s3[m][0]), "+v"(s3[m][1]));
    asm volatile("" : "+v"(lsum), "+v"(db3a));
    if constexpr (!SB) {
      if (ps + G < npass) stage(par ^ 1, tdv);
    }
    stamp(7);
    __syncthreads();  // B4: dZ2 complete, next pass's X / y staged (KT1 = 1)
    if constexpr (SB) {
      // (pass ps + G is prefetched after the dH1 stream below: its 8 X VGPRs not live there)
    } else if (ps + 2 * G < npass) {
      prefetch(ps + 2 * G, tdv);
      if (ps + 3 * G < npass) fetch_ids(ps + 3 * G, tdv);
    }
    stamp(8);

    stamp(9);
    // ---- dH1^T (own units k, K = 256 output units) = W2^T dZ2^T: stream steps 8..15
#pragma unroll
    for (int n = 0; n < NR; ++n) hb[n] = *reinterpret_cast<const bf16x8*>(zs + tile_off(16 * n + l15, 8 * g));
    w2z = 0;
    asm volatile("" : "+s"(w2z));
    static_for<0, 8>([&](auto kc) {
      constexpr int kt = decltype(kc)::value;
#pragma unroll
      for (int n = 0; n < NR; ++n) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[(8 + kt) % WD][m], hb[n],
                                                              kt == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[m][n], 0, 0, 0);
        if constexpr (kt + 1 < 8) {
          __builtin_amdgcn_sched_barrier(0);
          hb[n] = *reinterpret_cast<const bf16x8*>(zs + tile_off(16 * n + l15, 32 * (kt + 1) + 8 * g));
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // refill: W2^T steps 8 + kt + WD while they last, then the next pass's first W2 steps
#pragma unroll
      for (int m = 0; m < MT; ++m) wr[(8 + kt) % WD][m] = wfrag((8 + kt + WD) & 15, m);
    });
    if constexpr (SB) {
      if (ps + G < npass) {
        prefetch(ps + G, tdv);
        if (ps + 2 * G < npass) fetch_ids(ps + 2 * G, tdv);
      }
    }
    // global stores only after the next pass's W2 requests (vmcnt counts stores, in order)
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (pgr[q] >= 0 && pred != nullptr) pred[pgr[q]] = pst[q];
    stamp(10);
    // ---- dZ1 = bf16(dH1) where H1 > 0, over the same 8 bytes of h1s (rows past B: dZ2 = 0 there,
    // so dH1 and dZ1 are zero without a row test)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        uint2* pp = reinterpret_cast<uint2*>(h1s + tile_off(16 * n + l15, u0 + 16 * m + 4 * g));
        const uint2 hv = *pp;
        const unsigned o0 = mask_pk(pk_bf16(acc[m][n][0], acc[m][n][1]), hv.x);
        const unsigned o1 = mask_pk(pk_bf16(acc[m][n][2], acc[m][n][3]), hv.y);
        *pp = make_uint2(o0, o1);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    stamp(11);
    // ---- dW1^T slice (32 units x Fp) += dZ1^T X over the pass's 128 rows; db1 += dZ1^T 1. The
    // dZ2 copy-out as dW2 A fragments rides along (fragment (S, b) = 32 rows x 16 units; wave w
    // writes the pass's 4 row groups of its own unit blocks 2w, 2w + 1, two per K step, and sums
    // each fragment's rows into db2 with one MFMA against the ones operand): here the dH1
    // accumulators are dead, the next pass's W2 requests are out (vmcnt counts stores, in order),
    // and the stores overlap MFMAs — as a phase of its own after B4 it cost 2.4k cycles per pass
    // (tools/mlp_timeline.py). Rows past B hold zeros in zs (summed, store skipped)
    bf16x8 onesv = ones;
    asm volatile("" : "+v"(onesv));  // one 4-VGPR copy (left alone the splat was rebuilt per MFMA)
#pragma unroll
    for (int kk = 0; kk < R / 32; ++kk) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {  // copy-out fragments 2kk, 2kk + 1: unit block 2w + qq, rows 32kk..
        const int b = 2 * wid + qq;
        bf16x8 v;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bf16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(zs + tile_off(32 * kk + 8 * g + 4 * h + tq, 16 * b + 4 * tp)));
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * h + e] = t[e];
        }
        db2a[qq] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v, onesv, db2a[qq], 0, 0, 0);
        if (row0 + 32 * kk < B) {
          const size_t S = (size_t)(row0 >> 5) + kk;
          *reinterpret_cast<bf16x8*>(dZ2 + ((S * 16 + b) * 64 + lnv) * 8) = v;
        }
      }
      bf16x8 af[MT], bfr[NFT];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 32 * kk + 8 * g + 4 * h + tq;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(h1s + tile_off(r, u0 + 16 * m + 4 * tp)));
#pragma unroll
          for (int e = 0; e < 4; ++e) af[m][4 * h + e] = v[e];
        }
#pragma unroll
        for (int f = 0; f < NFT; ++f) {
          const int f0 = 16 * f + 4 * tp;
          const bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(xt + x_off<XW>(r, f0 >> 3) + ((f0 & 7) << 1)));
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[f][4 * h + e] = v[e];
        }
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
#pragma unroll
        for (int f = 0; f < NFT; ++f)
          dw1a[m][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[f], dw1a[m][f], 0, 0, 0);
        db1a[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], onesv, db1a[m], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    stamp(12);
  }

  // ---- batch sums -> copy blockIdx % kMlpRedCopies of the scratch; dW1 -> this workgroup's row.
  // db1 / db2: every column of the ones-MFMA accumulators holds the same sums (lanes l15 == 0)
  float* rb = red + (blockIdx.x & (kMlpRedCopies - 1)) * kMlpRedRow;
  float* slab = red + kMlpRedSlabOff + (size_t)blockIdx.x * kMlpRedSlabRow;
  const float tl = block_sum<512>(lsum, lred);
  if (tid == 0 && tl != 0.f) atomicAdd(rb + kMlpRedLoss, tl);
  const float t3 = block_sum<512>(db3a, lred);
  if (tid == 0 && t3 != 0.f) atomicAdd(rb + kMlpRedDb3, t3);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int u = u0 + 16 * m + 4 * g + r;
      float v = s3[m][r >> 1][r & 1];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if (l15 == 0) {
        if (v != 0.f) atomicAdd(rb + kMlpRedDw3 + u, v);
        if (db1a[m][r] != 0.f) atomicAdd(rb + kMlpRedDb1 + u, db1a[m][r]);
        if (db2a[m][r] != 0.f) atomicAdd(rb + kMlpRedDb2 + u, db2a[m][r]);
      }
    }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int f = 0; f < NFT; ++f) {
      const int ft = l15 + 16 * f;
      if (ft < Fp)
#pragma unroll
        for (int i = 0; i < 4; ++i) slab[(u0 + 16 * m + 4 * g + i) * Fp + ft] = dw1a[m][f][i];
    }
}

// ----------------------------------------------------------------------------------------
// dW2 [256 out][256 in] += dZ2^T H1, H1 = relu(X W1^T + b1) recomputed. dZ2 arrives in the
// fragment layout written by mlp2_step_kernel<., true> (fragment (S, b) = rows 32S .. 32S + 31
// x units 16b .. 16b + 15, 1 KiB, lane (l15, g) = rows 32S + 8g + j of unit 16b + l15), so a
// fragment is ONE 1-KiB LDS-DMA wave-instruction in and ONE conflict-free ds_read_b128 out.
// H1 is recomputed straight into the B-operand layout: the recompute MFMA's A operand (X rows)
// takes its 16 rows in the order 8(i >> 2) + 4h + (i & 3), so output lane (l15, g) holds rows
// 8g + 4h + r of unit l15 — exactly the K = rows slots of the dW MFMA's B fragment (no
// transpose, no H1 image in LDS: the LDS-staged mlp2_dw2_kernel spent its time writing that
// image, 16 % bank conflicts).
//  * (round 4, mlp2_dw2f_kernel: 256 (out) x 128 (in) tiles, 32 fragments per chunk; round 5:
//    mlp2_dw2g_kernel below, 128 x 256 tiles, 16 fragments per chunk.) Per 32-row step a wave
//    runs 4 recompute + 16 dW MFMAs (16x16x32).
//  * per 64-row chunk the workgroup DMAs its dZ2 fragments (2 per wave) + the 4-KiB X tile
//    (waves 0-3, one piece each, rows through the LDS row-id table) into a 4-slot ring, 3 chunks
//    ahead; one barrier per chunk. Fetches past the range re-load its last chunk (never read),
//    so every wave's DMA count per chunk is fixed and the vmcnt waits are immediates.
//  * grid = 2 tiles x nsplit row ranges; xcd_remap keeps a range's two tiles on one XCD, so
//    X (read by both tiles) hits L2 the second time.
constexpr int DW2F_MAX_ROWS = 2048;                      // rows per workgroup (the row-id table)

// ----------------------------------------------------------------------------------------
// dW2 from the fragment-layout dZ2 (the method above) with a 128 (out) x 256 (in) tile (round
// 5; round 4 used 256 x 128 tiles, mlp2_dw2f_kernel): wave w owns in columns 32w and all 128
// out rows, so a chunk needs only the 16 dZ2 fragments of the tile's out units (16 KiB of
// LDS-DMA instead of 32) and H1 is recomputed once per column (twice there); the MFMAs per
// (out, in) element and their order are unchanged (bit-identical dW2), +0.4 % step rate.
constexpr int DW2G_SLOTS = 6;  // 5 chunks in flight (128 KiB of LDS with the row-id table)
constexpr int DW2G_ABYTES = 16 * 1024;                  // 2 steps x 8 dZ2 fragments
// + the X tile [64 rows][32 KT1 bf16]. KT1 = 2 (Fp <= 64, round 6): 128-B rows (6 slots: 152 KiB
// of LDS with the row-id table), every wave DMAs one 8-row X piece per chunk, and the recompute
// runs two K steps; chunk c of row r at slot c ^ (((r >> 1) & 1) | ((r >> 2) & 6)) (the rows one
// ds_read_b128 lane group reads land on 16 distinct 16-B slots)
template <int KT1>
constexpr int dw2g_slot() { return DW2G_ABYTES + MF_ROWS * 64 * KT1; }
template <int KT1>
__global__ __launch_bounds__(512, 1) void mlp2_dw2g_kernel(const bf16_t* __restrict__ dZ2F, const bf16_t* __restrict__ X,
                                                           int Fp, const long long* __restrict__ rows, long nrows,
                                                           const bf16_t* __restrict__ W1, const float* __restrict__ b1,
                                                           int kchunk, float* __restrict__ dW2, float* __restrict__ slab,
                                                           int slab_row0, int prio) {
  constexpr int DW2G_SLOT = dw2g_slot<KT1>(), XW = 64 * KT1;
  __shared__ __attribute__((aligned(16))) char smem[DW2G_SLOTS * DW2G_SLOT + DW2F_MAX_ROWS * 4];
  int* ridx = reinterpret_cast<int*>(smem + DW2G_SLOTS * DW2G_SLOT);
  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool xw = KT1 == 2 || wid < 4;  // this wave also DMAs one X piece per chunk
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L >> 1, t = L & 1;
  const int o0 = 128 * t, n0 = 32 * wid;
  const int kbeg = split * kchunk, nch = kchunk / MF_ROWS;
  for (int i = tid; i < kchunk; i += 512) ridx[i] = rows != nullptr ? (int)data_row(rows, kbeg + i, nrows) : kbeg + i;
  __syncthreads();
  if (prio && wid >= 4) __builtin_amdgcn_s_setprio(1);

  bf16x8 w1f[2][KT1];
  float bias[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int u = n0 + 16 * nb + l15;
#pragma unroll
    for (int k = 0; k < KT1; ++k) {
      const int f = 32 * k + 8 * g;
      w1f[nb][k] = f + 8 <= Fp ? *reinterpret_cast<const bf16x8*>(W1 + (size_t)u * Fp + f) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    bias[nb] = b1[u];
  }
  auto xswz = [](int r) { return KT1 == 1 ? (r >> 3) & 3 : ((r >> 1) & 1) | ((r >> 2) & 6); };
  // DMA sources. dZ2 fragments (S, b) of the tile: b = 8t + mb; wave w moves (step w >> 2,
  // blocks 8t + 2 (w & 3) + {0, 1})
  const bf16_t* zsrc = dZ2F + ((size_t)(kbeg >> 5) * 16 + 8 * t + 2 * (wid & 3)) * 512 + lane * 8;
  // X piece of this wave: KT1 = 1 rows 16w + lane / 4 (waves 0-3), KT1 = 2 rows 8w + lane / 8;
  // lane = the LDS slot, loading the chunk stored there (chunks past Fp: chunk 0, times zero W1)
  const int xrow = KT1 == 1 ? 16 * (wid & 3) + (lane >> 2) : 8 * wid + (lane >> 3);
  int xq = (lane & (4 * KT1 - 1)) ^ xswz(xrow);
  if (8 * xq + 8 > Fp) xq = 0;
  auto issue = [&](int c, int slot) {
    char* st = smem + slot * DW2G_SLOT;
    const int s2 = wid >> 2;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bf16_t* src = zsrc + ((size_t)(2 * c + s2) * 16 + k) * 512;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(st + (s2 * 8 + 2 * (wid & 3) + k) * 1024), 16, 0, 0);
    }
    if (xw) {
      const size_t xr = (size_t)ridx[c * MF_ROWS + xrow];
      __builtin_amdgcn_global_load_lds((const void*)(X + xr * Fp + 8 * xq), (lds_void*)(st + DW2G_ABYTES + wid * 1024), 16, 0, 0);
    }
  };
  auto dma_wait = [&](auto nc) {
    constexpr int n = decltype(nc)::value;
    if (xw)
      wait_vmcnt<3 * n>();
    else
      wait_vmcnt<2 * n>();
  };
  int xg[KT1];
#pragma unroll
  for (int k = 0; k < KT1; ++k) xg[k] = 8 * (g + 4 * k) + 8 <= Fp ? g + 4 * k : 0;
  const int xr0 = 8 * (l15 >> 2) + (l15 & 3);

  f32x4 acc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int last = nch - 1;
#pragma unroll
  for (int k = 0; k < DW2G_SLOTS - 1; ++k) issue(min(k, last), k);
  for (int c = 0; c < nch; ++c) {
    const int slot = c % DW2G_SLOTS;
    dma_wait(std::integral_constant<int, DW2G_SLOTS - 2>{});  // chunk c's pieces (this wave) landed
    __builtin_amdgcn_s_barrier();                              // ... every wave's; slot c - 1 free
    asm volatile("" ::: "memory");
    issue(min(c + DW2G_SLOTS - 1, last), (c + DW2G_SLOTS - 1) % DW2G_SLOTS);
    const char* st = smem + slot * DW2G_SLOT;
    bf16x8 xfa[2][2][KT1], afa[2][8];
    auto frags = [&](int s2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 32 * s2 + xr0 + 4 * h;
#pragma unroll
        for (int k = 0; k < KT1; ++k)
          xfa[s2][h][k] = *reinterpret_cast<const bf16x8*>(st + DW2G_ABYTES + r * XW + ((xg[k] ^ xswz(r)) << 4));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mb = 0; mb < 8; ++mb)
        afa[s2][mb] = *reinterpret_cast<const bf16x8*>(st + (s2 * 8 + mb) * 1024 + lane * 16);
    };
    frags(0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 hb[2];
      const bf16x8(&xf)[2][KT1] = xfa[s2];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        // b1 as the C operand and the ReLU on the packed pair: the step kernel's H1, bit for bit
        // (the same K-step order)
        const f32x4 bc{bias[nb], bias[nb], bias[nb], bias[nb]};
        f32x4 c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[0][0], w1f[nb][0], bc, 0, 0, 0);
        f32x4 c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[1][0], w1f[nb][0], bc, 0, 0, 0);
        if constexpr (KT1 == 2) {
          c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[0][1], w1f[nb][1], c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[1][1], w1f[nb][1], c1, 0, 0, 0);
        }
        const unsigned p0 = relu_pk(pk_bf16(c0[0], c0[1]));
        const unsigned p1 = relu_pk(pk_bf16(c0[2], c0[3]));
        const unsigned p2 = relu_pk(pk_bf16(c1[0], c1[1]));
        const unsigned p3 = relu_pk(pk_bf16(c1[2], c1[3]));
        typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
        hb[nb] = __builtin_bit_cast(bf16x8, (u32x4_t{p0, p1, p2, p3}));
      }
      if (s2 == 0) {
        __builtin_amdgcn_sched_barrier(0);
        frags(1);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afa[s2][mb], hb[nb], acc[mb][nb], 0, 0, 0);
      }
    }
  }
  wait_vmcnt<0>();  // the clamped fetches past the range must land before the workgroup ends
  const int srow = slab_row0 + split;
  if (srow < kMlpRedSlab2Rows) {
    float* dst = slab + (size_t)srow * 65536;
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) dst[(size_t)(o0 + 16 * mb + 4 * g + r) * MF_H + n0 + 16 * nb + l15] = acc[mb][nb][r];
  } else {
    float* dst = dW2 + (size_t)(split & (kMlpRedCopies2 - 1)) * 65536;
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          atomicAdd(dst + (size_t)(o0 + 16 * mb + 4 * g + r) * MF_H + n0 + 16 * nb + l15, acc[mb][nb][r]);
  }
}
}  // namespace

bool launch_mlp2_step(const bf16_t* X, int Fp, const bf16_t* W1, const float* b1, const bf16_t* W2, const float* b2,
                      const float* w3, const float* b3, const float* y, float dy_scale, int B, const long long* rows,
                      long nrows, bf16_t* dZ2, float* pred, float* red, bool dz_frag, hipStream_t s,
                      const bf16_t* W2T, float clip) {
  // the reduce sums the dW1 rows only when it expects the 8-wave backward's layout
  if (B <= 0 || Fp > 64 || Fp % 8 != 0 || red == nullptr || !mlp_bwd8()) return false;
  if (dz_frag && B % MF_ROWS != 0) return false;
  if (Fp > 32 && (W2T == nullptr || !dz_frag)) return false;  // Fp <= 64: the 128-row kernel only
  const int grid = mlp2_train_grid(B);  // the dW1 rows mlp2_reduce sums
  // phase stamps (tools/mlp_timeline.py; results unchanged, so not a WF_DIAG-only switch):
  // into dW2 slab rows 200.. of the scratch (unused by a step of <= 200 dW2 ranges)
  static const bool stamp = diag_env_int("WELLFLOW_MLP_STAMP", 0) != 0;  // WF_DIAG builds only
  // static s_setprio 1 for waves 4-7 (+0.2 to +1.1 % in three interleaved pairs, chunk span
  // 17.5k -> 17.1k cycles, profiles/r4/mlp_prio; the WELLFLOW_STEP_PRIO A/B knob was removed)
  constexpr int prio = 1;
  if (W2T != nullptr && dz_frag) {  // 128-row passes, both weight images streamed
    if (rows != nullptr && nrows > 0x7FFFFFFFL) return false;  // 32-bit row ids in the kernel
    // the same static priority split for the 128-row kernel (A/B: WELLFLOW_MLP_PRIO128, WF_DIAG only)
    static const int prio128 = diag_env_int("WELLFLOW_MLP_PRIO128", prio);
    if (stamp && Fp <= 16) {
      hipLaunchKernelGGL((mlp2_step128_kernel<1, true>), dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, W2T, b2, w3, b3,
                         y, dy_scale, clip, B, rows, nrows, dZ2, pred, red, prio128,
                         reinterpret_cast<unsigned long long*>(red + kMlpRedSlab2Off + 200L * 65536));
      return true;
    }
    if (Fp <= 16)
      hipLaunchKernelGGL(mlp2_step128_kernel<1>, dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, W2T, b2, w3, b3, y,
                         dy_scale, clip, B, rows, nrows, dZ2, pred, red, prio128);
    else if (Fp <= 32)
      hipLaunchKernelGGL(mlp2_step128_kernel<2>, dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, W2T, b2, w3, b3, y,
                         dy_scale, clip, B, rows, nrows, dZ2, pred, red, prio128);
    else
      hipLaunchKernelGGL(mlp2_step128_kernel<4>, dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, W2T, b2, w3, b3, y,
                         dy_scale, clip, B, rows, nrows, dZ2, pred, red, prio128);
    return true;
  }
  if (stamp && Fp <= 16 && dz_frag) {
    hipLaunchKernelGGL((mlp2_step_kernel<1, true, true>), dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y,
                       dy_scale, clip, B, rows, nrows, dZ2, pred, red, prio,
                       reinterpret_cast<unsigned long long*>(red + kMlpRedSlab2Off + 200L * 65536));
    return true;
  }
#define WF_STEP(NFT, FR)                                                                                            \
  hipLaunchKernelGGL((mlp2_step_kernel<NFT, FR>), dim3(grid), dim3(512), 0, s, X, Fp, W1, b1, W2, b2, w3, b3, y, \
                     dy_scale, clip, B, rows, nrows, dZ2, pred, red, prio)
  if (Fp <= 16) {
    if (dz_frag) WF_STEP(1, true); else WF_STEP(1, false);
  } else {
    if (dz_frag) WF_STEP(2, true); else WF_STEP(2, false);
  }
#undef WF_STEP
  return true;
}

// dW2 (the spread scratch's dW2 copies: red + kMlpRedCopies * kMlpRedRow) from the fragment-
// layout dZ2; B % 64 == 0, Fp <= 64. nsplit row ranges (<= 128: two tiles per range, one
// workgroup per CU); batches beyond 128 ranges of DW2F_MAX_ROWS rows run as consecutive
// launches over row blocks. False = not covered.
int launch_mlp2_dw2f(const bf16_t* dZ2F, const bf16_t* X, int Fp, const long long* rows, long nrows, const bf16_t* W1,
                     const float* b1, int B, int nsplit, float* red, hipStream_t s) {
  if (B <= 0 || B % MF_ROWS != 0 || Fp > 64 || Fp % 8 != 0 || red == nullptr) return 0;
  constexpr int kMaxBlock = 128 * DW2F_MAX_ROWS;  // rows per launch
  // static s_setprio 1 for waves 4-7 (48.2 -> 47.0 us, +0.3 to +0.6 % in three interleaved pairs,
  // profiles/r4/mlp_prio; the WELLFLOW_DW2F_PRIO A/B knob was removed)
  constexpr int prio = 1;
  int srow = 0;  // slab rows used so far (the launches' ranges stack)
  for (int r0 = 0; r0 < B; r0 += kMaxBlock) {
    const int Bb = B - r0 < kMaxBlock ? B - r0 : kMaxBlock;
    const int chunks = Bb / MF_ROWS;
    int ns = nsplit < 1 ? 1 : (nsplit > 128 ? 128 : nsplit);
    while (ns < 128 && (chunks + ns - 1) / ns * MF_ROWS > DW2F_MAX_ROWS) ++ns;
    while (ns > 1 && chunks % ns != 0) --ns;
    const int kchunk = (chunks / ns) * MF_ROWS;
    if (kchunk > DW2F_MAX_ROWS) return 0;  // (unreachable for B % 64 == 0)
    // row block r0: dZ2 fragments start at step r0 / 32; X through `rows` (offset) or directly
    hipLaunchKernelGGL(Fp <= 32 ? mlp2_dw2g_kernel<1> : mlp2_dw2g_kernel<2>, dim3(2 * ns), dim3(512), 0, s, dZ2F + (size_t)r0 * MF_H,
                       rows != nullptr ? X : X + (size_t)r0 * Fp, Fp, rows != nullptr ? rows + r0 : nullptr,
                       rows != nullptr ? nrows : (long)Bb, W1, b1, kchunk, red + (size_t)kMlpRedCopies * kMlpRedRow,
                       red + kMlpRedSlab2Off, srow, prio);
    srow += ns;
  }
  return srow < kMlpRedSlab2Rows ? srow : kMlpRedSlab2Rows;
}


}  // namespace wf
