// wellflow — general MFMA GEMM with fused epilogues (gfx950).
//
//   out[m, n] = act(alpha * sum_k A(m,k) B(n,k) + beta * out[m, n] + bias[n]) (* mask)
//
// Used by the static / dynamic MLP (GEMM + bias + ReLU forward,
// dX with the ReLU-mask epilogue, dW = dZ^T X with MN-contiguous operands), the CNN
// (K1/K5/K7) and the LSTM weight gradient (K14). Split-K reduces through fp32 atomics
// into the (pre-zeroed) fp32 output: the weight-gradient GEMMs here have tiny M x N
// (<= 2048 x 576) and a huge K (batch x time), so the atomic bytes are <1% of the
// MFMA time (cdna_hip_programming.md Guideline 12 sizing rule).
#include <cstdlib>

#include "gemm_core.h"
#include "kernels.h"

namespace wf {

// dropout stream of this launch: the host seed, mixed with the device step counter when one
// is given (so a hipGraph replay draws a fresh mask every step)
__device__ __forceinline__ unsigned long long drop_seed(const GemmEpilogue& e) {
  return e.seed_dev != nullptr ? e.seed ^ ((unsigned long long)e.seed_dev[0] * 0xD1B54A32D192ED03ull) : e.seed;
}

// STAGES >= 2: direct-to-LDS ring; the host only selects it when every K chunk is a
// multiple of 64 and the whole-tile over-read past M / N stays inside the operand
// allocations (binding.cpp computes that from the tensor sizes); results outside M x N
// are discarded by the epilogue as in the register path.
template <int BM, int BN, int LA, int LB, int STAGES, int WM = 2, int WN = 2>
__global__ __launch_bounds__(64 * WM * WN) void gemm_kernel(const bf16_t* __restrict__ A, long lda,
                                                   const bf16_t* __restrict__ B, long ldb,
                                                   int M, int N, int K, int kchunk,
                                                   GemmEpilogue e) {
  using C = GemmCfg<BM, BN, LA, LB, WM, WN>;
  constexpr int LDSB = STAGES * C::STAGE > C::LDS_BYTES ? STAGES * C::STAGE : C::LDS_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  const int tiles_n = (N + BN - 1) / BN;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, t = L % tiles;
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int kbeg = split * kchunk;
  const int kend = min(K, kbeg + kchunk);

  f32x4 acc[C::TM][C::TN];
  if constexpr (STAGES >= 2)
    gemm_mainloop_glds2<C, STAGES>(A, lda, B, ldb, kbeg, (kend - kbeg) / 64, m0, n0, smem, acc);
  else
    gemm_mainloop<C>(A, lda, M, B, ldb, N, kbeg, kend, m0, n0, smem, acc);

  const AccCoord<C> cc(m0, n0);

  // Staged bf16 epilogue: the ReLU-mask tile is read and the bf16 output tile written
  // through LDS ([BM][BN] bf16 each, 16-B chunks XOR-swizzled by row) so global traffic is
  // whole 16-B-per-lane row segments instead of 2-B scattered accesses.
  static_assert(2 * BM * BN * 2 <= LDSB, "staging tiles must fit the mainloop LDS");
  const bool staged = e.stage_ok && e.outH != nullptr && e.outF == nullptr && !e.atomic;
  if (staged) {
    constexpr int CPR = BN / 8;  // 16-B chunks per tile row
    bf16_t* mt = reinterpret_cast<bf16_t*>(smem);
    bf16_t* ot = reinterpret_cast<bf16_t*>(smem + BM * BN * 2);
    auto chunk_off = [&](int row, int c8) { return row * BN + ((c8 ^ (row & (CPR - 1))) << 3); };
    if (e.mask != nullptr) {
      for (int q = threadIdx.x; q < BM * CPR; q += C::NT) {
        const int row = q / CPR, c8 = q % CPR;
        const int m = m0 + row, n = n0 + c8 * 8;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (m < M && n < N) v = *reinterpret_cast<const uint4*>(e.mask + (size_t)m * e.ldm + n);
        *reinterpret_cast<uint4*>(mt + chunk_off(row, c8)) = v;
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int n = cc.col(j);
      const int col = n - n0;
      const bool nok = n < N;
      const float bn = (e.bias != nullptr && nok) ? e.bias[n] : 0.f;
      float csum = 0.f;
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = cc.row(i, r);
          const int row = m - m0;
          const int lo = chunk_off(row, col >> 3) + (col & 7);
          float v = e.alpha * acc[i][j][r] + bn;
          if (e.act == 1) v = fmaxf(v, 0.f);
          if (e.drop_p > 0.f)
            v = uniform_hash(drop_seed(e), (unsigned long long)m * N + n) >= e.drop_p
                    ? v * (1.f / (1.f - e.drop_p)) : 0.f;
          if (e.mask != nullptr) v = bf2f(mt[lo]) > 0.f ? v * e.mask_scale : 0.f;
          const bf16_t vb = f2bf(v);
          ot[lo] = vb;
          if (nok && m < M) csum += bf2f(vb);
        }
      }
      if (e.colsum != nullptr) {
        csum += __shfl_xor(csum, 16, 64);
        csum += __shfl_xor(csum, 32, 64);
        if ((threadIdx.x & 63) < 16 && nok) atomicAdd(e.colsum + n, csum);
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < BM * CPR; q += C::NT) {
      const int row = q / CPR, c8 = q % CPR;
      const int m = m0 + row, n = n0 + c8 * 8;
      if (m < M && n < N)
        *reinterpret_cast<uint4*>(e.outH + (size_t)m * e.ldo + n) =
            *reinterpret_cast<const uint4*>(ot + chunk_off(row, c8));
    }
    return;
  }

#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    const int n = cc.col(j);
    const bool nok = n < N;
    const float bn = (e.bias != nullptr && nok) ? e.bias[n] : 0.f;
    float csum = 0.f;
#pragma unroll
    for (int i = 0; i < C::TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = cc.row(i, r);
        if (!nok || m >= M) continue;
        float v = e.alpha * acc[i][j][r];
        const size_t o = (size_t)m * e.ldo + n;
        if (e.atomic) {
          atomicAdd(e.outF + o, v);
          continue;
        }
        if (e.beta != 0.f) v += e.beta * e.outF[o];
        v += bn;
        if (e.act == 1) v = fmaxf(v, 0.f);
        if (e.drop_p > 0.f)
          v = uniform_hash(drop_seed(e), (unsigned long long)m * N + n) >= e.drop_p
                  ? v * (1.f / (1.f - e.drop_p)) : 0.f;
        if (e.mask != nullptr)
          v = bf2f(e.mask[(size_t)m * e.ldm + n]) > 0.f ? v * e.mask_scale : 0.f;
        csum += v;
        if (e.outF != nullptr) e.outF[o] = v;
        if (e.outH != nullptr) e.outH[o] = f2bf(v);
      }
    }
    if (e.colsum != nullptr) {
      csum += __shfl_xor(csum, 16, 64);
      csum += __shfl_xor(csum, 32, 64);
      if ((threadIdx.x & 63) < 16 && nok) atomicAdd(e.colsum + n, csum);
    }
  }
}

template <int BM, int BN, int LA, int LB>
static void launch_cfg(const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N, int K,
                       int ksplit, const GemmEpilogue& e, hipStream_t s, bool glds_ok) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (ksplit < 1) ksplit = 1;
  int kchunk = (K + ksplit - 1) / ksplit;
  kchunk = (kchunk + 63) / 64 * 64;
  if (kchunk < 64) kchunk = 64;
  const int nsplit = (K + kchunk - 1) / kchunk;
  const dim3 grid(tiles * (nsplit > 0 ? nsplit : 1));
  if (glds_ok && K % 64 == 0)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB, 3>), grid, dim3(256), 0, s, A, lda, B, ldb, M,
                       N, K, kchunk, e);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, LA, LB, 0>), grid, dim3(256), 0, s, A, lda, B, ldb, M,
                       N, K, kchunk, e);
}

// Big-tile configuration for the MN x MN weight-gradient GEMMs (dW = dZ^T X over a huge
// batch/time K): 256x128 tile, 8 waves, 3-stage glds ring (144 KiB): 87 FLOP per staged
// byte instead of 64 for 128x128.
static void launch_dw_big(const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N, int K,
                          int ksplit, const GemmEpilogue& e, hipStream_t s) {
  constexpr int BM = 256, BN = 128;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int kchunk = ((K + ksplit - 1) / ksplit + 63) / 64 * 64;
  const int nsplit = (K + kchunk - 1) / kchunk;
  hipLaunchKernelGGL((gemm_kernel<BM, BN, MN_CONTIG, MN_CONTIG, 3, 4, 2>), dim3(tiles * nsplit),
                     dim3(512), 0, s, A, lda, B, ldb, M, N, K, kchunk, e);
}

// LSTM weight gradient (M = 4H = 2048, N = KA = 576, K = T*B), alternative tile: 128x288,
// 4 waves of 64x144, 3-stage ring (156 KiB). N = 2 x 288 exactly (the 256x128 tile wastes
// half of its 5th column tile) and 16 x 2 = 32 tiles per K split = one XCD's 32 CUs. Measured
// slower than the 256x128 8-wave tile (1.60 vs 1.33 ms at split-K 32: one wave per SIMD
// cannot hide the fragment reads), so it is opt-in (WELLFLOW_DW_BIG=2).
// Split-K weight-gradient kernel: MN x MN operands, full tiles only (M % BM == N % BN == 0,
// host-checked), epilogue = fp32 atomic add of alpha * acc (nothing else, so the 144
// accumulator registers stay in registers).
template <int BM, int BN, int STAGES, int WM, int WN, int PRIO = 0>
__global__ __launch_bounds__(64 * WM * WN) void gemm_dw_kernel(const bf16_t* __restrict__ A, long lda,
                                                      const bf16_t* __restrict__ B, long ldb, int N,
                                                      int kchunk, int tiles, float* __restrict__ out,
                                                      long ldo, float alpha) {
  using C = GemmCfg<BM, BN, MN_CONTIG, MN_CONTIG, WM, WN>;
  __shared__ __attribute__((aligned(16))) char smem[STAGES * C::STAGE];
  const int tiles_n = N / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, t = L % tiles;
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  f32x4 acc[C::TM][C::TN];
  gemm_mainloop_glds2<C, STAGES, PRIO>(A, lda, B, ldb, split * kchunk, kchunk / 64, m0, n0, smem, acc);
  const AccCoord<C> cc(m0, n0);
#pragma unroll
  for (int j = 0; j < C::TN; ++j)
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        atomicAdd(out + (size_t)cc.row(i, r) * ldo + cc.col(j), alpha * acc[i][j][r]);
}

static void launch_dw_288(const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N, int K,
                          int ksplit, const GemmEpilogue& e, hipStream_t s) {
  constexpr int BM = 128, BN = 288;
  const int tiles = (M / BM) * (N / BN);
  // equal 64-aligned K chunks (K % (64 * nsplit) == 0 is required: partial chunks would need
  // the masked mainloop)
  int nsplit = ksplit;
  while (nsplit > 1 && K % (64 * nsplit) != 0) --nsplit;
  const int kchunk = K / nsplit;
  hipLaunchKernelGGL((gemm_dw_kernel<BM, BN, 3, 2, 2>), dim3(tiles * nsplit), dim3(256), 0, s, A, lda, B, ldb,
                     N, kchunk, tiles, e.outF, e.ldo, e.alpha);
}

// 256x192, 8 waves of 64x96, 2-stage ring (112 KiB): N = 576 = 3 x 192 exactly, and 22 % fewer
// operand bytes per MFMA than 256x128 (rotation-swizzled 192-wide MN image).
static void launch_dw_192(const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N, int K,
                          int ksplit, const GemmEpilogue& e, hipStream_t s) {
  constexpr int BM = 256, BN = 192;
  const int tiles = (M / BM) * (N / BN);
  int nsplit = ksplit;
  while (nsplit > 1 && K % (64 * nsplit) != 0) --nsplit;
  const int kchunk = K / nsplit;
  // s_setprio(1) around each MFMA cluster (cdna_hip_programming.md §5.5 T5: hipcc then keeps
  // the clusters between the barriers): 1.24 -> 1.16 ms at B = 8192 (WELLFLOW_DW_PRIO=0/2: off /
  // static priority for waves 4-7, no gain)
  constexpr int prio = 1;  // WELLFLOW_DW_PRIO=0/2 measured no gain (round 2): knob removed in round 5
  if (prio == 1)
    hipLaunchKernelGGL((gemm_dw_kernel<BM, BN, 2, 4, 2, 1>), dim3(tiles * nsplit), dim3(512), 0, s, A, lda, B, ldb,
                       N, kchunk, tiles, e.outF, e.ldo, e.alpha);
  else if (prio == 2)
    hipLaunchKernelGGL((gemm_dw_kernel<BM, BN, 2, 4, 2, 2>), dim3(tiles * nsplit), dim3(512), 0, s, A, lda, B, ldb,
                       N, kchunk, tiles, e.outF, e.ldo, e.alpha);
  else
    hipLaunchKernelGGL((gemm_dw_kernel<BM, BN, 2, 4, 2>), dim3(tiles * nsplit), dim3(512), 0, s, A, lda, B, ldb,
                       N, kchunk, tiles, e.outF, e.ldo, e.alpha);
}

// 256x192, 8 waves of 64x96, 32-deep half steps through an NSLOT-deep ring (gemm_core.h
// gemm_mainloop_glds_h): the same tile as launch_dw_192 with its DMA issued NSLOT - 1 half
// steps ahead instead of one 64-deep step
template <int BM, int BN, int NSLOT, int WM, int WN, int PRIO, int BKD = 32, bool GL = false, int DG = 0>
__global__ __launch_bounds__(64 * WM * WN) void gemm_dw_h_kernel(const bf16_t* __restrict__ A, long lda,
                                                        const bf16_t* __restrict__ B, long ldb, int N,
                                                        int kchunk, int tiles, float* __restrict__ out,
                                                        long ldo, float alpha, float* __restrict__ slab,
                                                        long slab_stride) {
  using C = GemmCfg<BM, BN, MN_CONTIG, MN_CONTIG, WM, WN>;
  constexpr int STAGE = (BM + BN) * BKD * 2;
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * STAGE];
  const int tiles_n = N / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, t = L % tiles;
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  f32x4 acc[C::TM][C::TN];
  gemm_mainloop_glds_h<C, NSLOT, PRIO, BKD, GL, DG>(A, lda, B, ldb, split * kchunk, kchunk / BKD, m0, n0, smem, acc);
  const AccCoord<C> cc(m0, n0);
  if (slab != nullptr) {  // this split's partial tile, plain-stored (dw_slab_reduce_kernel adds the splits)
    float* o = slab + (size_t)split * slab_stride;
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[(size_t)cc.row(i, r) * ldo + cc.col(j)] = alpha * acc[i][j][r];
    return;
  }
#pragma unroll
  for (int j = 0; j < C::TN; ++j)
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        atomicAdd(out + (size_t)cc.row(i, r) * ldo + cc.col(j), alpha * acc[i][j][r]);
}

// the same tile and 2-slot 64-deep ring as launch_dw_192, wave groups staggered by a barrier
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void gemm_dw_s_kernel(const bf16_t* __restrict__ A, long lda,
                                                        const bf16_t* __restrict__ B, long ldb, int N,
                                                        int kchunk, int tiles, float* __restrict__ out,
                                                        long ldo, float alpha) {
  using C = GemmCfg<BM, BN, MN_CONTIG, MN_CONTIG, WM, WN>;
  __shared__ __attribute__((aligned(16))) char smem[2 * C::STAGE];
  const int tiles_n = N / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, t = L % tiles;
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  f32x4 acc[C::TM][C::TN];
  gemm_mainloop_stag<C>(A, lda, B, ldb, split * kchunk, kchunk / 64, m0, n0, smem, acc);
  const AccCoord<C> cc(m0, n0);
#pragma unroll
  for (int j = 0; j < C::TN; ++j)
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        atomicAdd(out + (size_t)cc.row(i, r) * ldo + cc.col(j), alpha * acc[i][j][r]);
}

static void launch_dw_192h(const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N, int K,
                           int ksplit, int nslot, const GemmEpilogue& e, hipStream_t s) {
  constexpr int BM = 256, BN = 192;
  const int tiles = (M / BM) * (N / BN);
  int nsplit = ksplit;
  while (nsplit > 1 && K % (64 * nsplit) != 0) --nsplit;
  const int kchunk = K / nsplit;
  const dim3 grid(tiles * nsplit);
  if (nslot == 2)  // staggered wave groups (gemm_mainloop_stag)
    hipLaunchKernelGGL((gemm_dw_s_kernel<BM, BN, 4, 2>), grid, dim3(512), 0, s, A, lda, B, ldb, N, kchunk, tiles,
                       e.outF, e.ldo, e.alpha);
  else if (nslot == 5)
    hipLaunchKernelGGL((gemm_dw_h_kernel<BM, BN, 5, 4, 2, 1>), grid, dim3(512), 0, s, A, lda, B, ldb, N, kchunk,
                       tiles, e.outF, e.ldo, e.alpha, nullptr, 0L);
  else
    hipLaunchKernelGGL((gemm_dw_h_kernel<BM, BN, 4, 4, 2, 1>), grid, dim3(512), 0, s, A, lda, B, ldb, N, kchunk,
                       tiles, e.outF, e.ldo, e.alpha, nullptr, 0L);
}

// out[i] += sum over the nsplit slab slices (float4 per thread, all slice loads in flight)
__global__ __launch_bounds__(256) void dw_slab_reduce_kernel(float* __restrict__ out, const float* __restrict__ slab,
                                                             int nsplit, long n4) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float4* src = reinterpret_cast<const float4*>(slab) + i;
  float4 a = reinterpret_cast<float4*>(out)[i];
  for (int s0 = 0; s0 < nsplit; s0 += 8) {
    float4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = s0 + j < nsplit ? src[(size_t)(s0 + j) * n4] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a.x += v[j].x;
      a.y += v[j].y;
      a.z += v[j].z;
      a.w += v[j].w;
    }
  }
  reinterpret_cast<float4*>(out)[i] = a;
}

// 256x288, 8 waves of 64x144, 4-slot 32-deep ring (136 KiB; a 2-stage 64-deep ring spilled 61 VGPRs).
// Round 5: 4 waves of 128x144 (one per SIMD, accumulators in AGPRs; 35 % fewer LDS fragment
// reads) measured 1.18-1.25 vs 1.03 ms standalone (tools/dw_tiles.py, profiles/r5/notes.md): removed
// (default: 1.107 vs 1.166 ms for 256x192 standalone, 1.150 vs 1.178 ms inside the bench step): N = 576 = 2 x 288, 24 % more
// FLOP per staged byte than 256x192 (the dW loop's LDS-DMA bytes per CU per step, not its
// MFMAs or the DMA latency, track its time across tiles: 256x128 1.33, 256x192 1.17 ms)
static void launch_dw_288w(const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N, int K,
                           int ksplit, const GemmEpilogue& e, hipStream_t s, bool gl = false, int dg = 0) {
  constexpr int BM = 256, BN = 288;
  const int tiles = (M / BM) * (N / BN);
  // one workgroup per CU: 16 tiles x split-K 16 on 256 CUs (tools/dw_tiles.py, B = 8192:
  // split-K 16 / 32 / 64 = 1.107 / 1.115 / 1.160 ms)
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n;
  }();
  if (ksplit * tiles > cus && cus / tiles >= 1) ksplit = cus / tiles;
  int nsplit = ksplit;
  while (nsplit > 1 && K % (64 * nsplit) != 0) --nsplit;
  const int kchunk = K / nsplit;
  // split-K partials: fp32 atomics into the output (2048 x 576 x 16 splits = 75 MB of 64-B-segment
  // atomics at the tail of the kernel) or, given a slab, plain stores + one reduce
  const long mn = (long)M * N;
  const bool use_slab = e.slab != nullptr && e.ldo == N && nsplit > 1 && (long)nsplit * mn <= e.slab_cap && mn % 4 == 0;
  // s_setprio 1 around each MFMA cluster (static priority for waves 4-7 measured slower, r4/lstm_dw_prio;
  // the WELLFLOW_DW288_PRIO knob was removed in round 5)
  constexpr int prio = 1;
  if (dg == 1)  // tiles 9 / 10: diagnostics (wrong results), gemm_core.h gemm_mainloop_glds_h DG
    hipLaunchKernelGGL((gemm_dw_h_kernel<BM, BN, 4, 4, 2, 1, 32, false, 1>), dim3(tiles * nsplit), dim3(512), 0, s, A,
                       lda, B, ldb, N, kchunk, tiles, e.outF, e.ldo, e.alpha, use_slab ? e.slab : nullptr,
                       use_slab ? mn : 0L);
  else if (dg == 2)
    hipLaunchKernelGGL((gemm_dw_h_kernel<BM, BN, 4, 4, 2, 1, 32, false, 2>), dim3(tiles * nsplit), dim3(512), 0, s, A,
                       lda, B, ldb, N, kchunk, tiles, e.outF, e.ldo, e.alpha, use_slab ? e.slab : nullptr,
                       use_slab ? mn : 0L);
  else if (dg == 3)  // tile 11: DMA pieces between the MFMAs (gemm_core.h DG 3)
    hipLaunchKernelGGL((gemm_dw_h_kernel<BM, BN, 4, 4, 2, 1, 32, false, 3>), dim3(tiles * nsplit), dim3(512), 0, s, A,
                       lda, B, ldb, N, kchunk, tiles, e.outF, e.ldo, e.alpha, use_slab ? e.slab : nullptr,
                       use_slab ? mn : 0L);
  else if (gl)  // tile 8 (A/B): the DMA by global_load_lds; measured slower (1.105 vs 1.050 ms, r6/diag/glds.txt)
    hipLaunchKernelGGL((gemm_dw_h_kernel<BM, BN, 4, 4, 2, 1, 32, true>), dim3(tiles * nsplit), dim3(512), 0, s, A, lda,
                       B, ldb, N, kchunk, tiles, e.outF, e.ldo, e.alpha, use_slab ? e.slab : nullptr,
                       use_slab ? mn : 0L);
  else if (prio == 3)
    hipLaunchKernelGGL((gemm_dw_h_kernel<BM, BN, 4, 4, 2, 3, 32>), dim3(tiles * nsplit), dim3(512), 0, s, A, lda, B,
                       ldb, N, kchunk, tiles, e.outF, e.ldo, e.alpha, use_slab ? e.slab : nullptr, use_slab ? mn : 0L);
  else
    hipLaunchKernelGGL((gemm_dw_h_kernel<BM, BN, 4, 4, 2, 1, 32>), dim3(tiles * nsplit), dim3(512), 0, s, A, lda, B,
                       ldb, N, kchunk, tiles, e.outF, e.ldo, e.alpha, use_slab ? e.slab : nullptr, use_slab ? mn : 0L);
  if (use_slab) {
    const long n4 = mn / 4;
    hipLaunchKernelGGL(dw_slab_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, e.outF,
                       (const float*)e.slab, nsplit, n4);
  }
}

void launch_gemm(const bf16_t* A, long lda, int a_mn, const bf16_t* B, long ldb, int b_mn, int M,
                 int N, int K, int ksplit, const GemmEpilogue& e, hipStream_t s, bool glds_ok) {
  if (a_mn && b_mn && glds_ok && e.atomic && (e.big_tile >= 7 && e.big_tile <= 11) && M % 256 == 0 && K % 64 == 0) {
    if (N % 288 == 0) {
      launch_dw_288w(A, lda, B, ldb, M, N, K, ksplit < 1 ? 1 : ksplit, e, s, e.big_tile == 8,
                     e.big_tile >= 9 ? e.big_tile - 8 : 0);
      return;
    }
    if (N % 192 == 0) {  // e.g. H = 128 (KA = 192): the 256x192 tile
      launch_dw_192(A, lda, B, ldb, M, N, K, ksplit < 1 ? 1 : ksplit, e, s);
      return;
    }
  }
  // 4 / 5: the 256x192 tile with the 5- / 4-slot half-step ring; 6: staggered wave groups
  if (a_mn && b_mn && glds_ok && e.atomic && (e.big_tile >= 4 && e.big_tile <= 6) && M % 256 == 0 &&
      N % 192 == 0 && K % 64 == 0) {
    launch_dw_192h(A, lda, B, ldb, M, N, K, ksplit < 1 ? 1 : ksplit,
                   e.big_tile == 4 ? 5 : (e.big_tile == 5 ? 4 : 2), e, s);
    return;
  }
  if (a_mn && b_mn && glds_ok && e.atomic && e.big_tile == 2 && M % 128 == 0 && N % 288 == 0 && K % 64 == 0) {
    launch_dw_288(A, lda, B, ldb, M, N, K, ksplit < 1 ? 1 : ksplit, e, s);
    return;
  }
  if (a_mn && b_mn && glds_ok && e.atomic && e.big_tile == 3 && M % 256 == 0 && N % 192 == 0 && K % 64 == 0) {
    launch_dw_192(A, lda, B, ldb, M, N, K, ksplit < 1 ? 1 : ksplit, e, s);
    return;
  }
  if (a_mn && b_mn && glds_ok && e.atomic && e.big_tile && M % 256 == 0 && K % 64 == 0) {
    launch_dw_big(A, lda, B, ldb, M, N, K, ksplit < 1 ? 1 : ksplit, e, s);
    return;
  }
  if (!a_mn && !b_mn)
    launch_cfg<128, 128, K_CONTIG, K_CONTIG>(A, lda, B, ldb, M, N, K, ksplit, e, s, glds_ok);
  else if (!a_mn && b_mn)
    launch_cfg<128, 128, K_CONTIG, MN_CONTIG>(A, lda, B, ldb, M, N, K, ksplit, e, s, glds_ok);
  else if (a_mn && !b_mn)
    launch_cfg<128, 128, MN_CONTIG, K_CONTIG>(A, lda, B, ldb, M, N, K, ksplit, e, s, glds_ok);
  else
    launch_cfg<128, 128, MN_CONTIG, MN_CONTIG>(A, lda, B, ldb, M, N, K, ksplit, e, s, glds_ok);
}

}  // namespace wf
