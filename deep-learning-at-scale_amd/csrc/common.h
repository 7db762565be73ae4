// wellflow native kernel library — shared device helpers (gfx950 / CDNA4 only).
//
// Storage conventions used by every kernel in this library:
//   * bf16 tensors are raw 16-bit words (`bf16_t` = unsigned short); arithmetic is
//     always done in fp32 and converted with the helpers below.
//   * fp32 master weights / gradients / optimizer state live in flat buffers that
//     the Python side views as parameters (wellflow/optim/flat.py).
//   * wave64: every cross-lane idiom assumes 64 lanes (never 32).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include <cstdlib>

namespace wf {

typedef unsigned short bf16_t;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// Environment overrides of A/B variants and tuning sweeps: only WF_DIAG builds
// (WELLFLOW_DIAG_BUILD=1) read them; a production build compiles every such read to its
// default, so the set of WELLFLOW_* variables a production _C.so reads is exactly the
// documented list (README "Environment knobs", tests/test_diag_cpu.py).
inline int diag_env_int(const char* name, int dflt) {
#ifdef WF_DIAG
  const char* v = std::getenv(name);
  return v != nullptr ? std::atoi(v) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

__device__ __forceinline__ float bf2f(bf16_t x) {
  return __uint_as_float(static_cast<unsigned>(x) << 16);
}

// Round-to-nearest-even; a plain cast lowers to v_cvt_pk_bf16_f32 on gfx950 which
// keeps NaNs NaN (MI355X_MICROARCH.md, correctness boundaries).
__device__ __forceinline__ bf16_t f2bf(float x) {
  __hip_bfloat16 h = __float2bfloat16(x);
  return *reinterpret_cast<bf16_t*>(&h);
}

// Two floats -> one packed bf16 pair (lo in bits 0-15): a single v_cvt_pk_bf16_f32 (RNE),
// where f2bf(a) | f2bf(b) << 16 costs two conversions plus the and / shift / or to merge.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t{lo, hi}), bf16x2_t));
}

// Gate activations on the transcendental unit: v_exp_f32 + v_rcp_f32 (1 ulp), no IEEE
// division sequence (the precise 1/x costs ~10 VALU and dominated the LSTM epilogues).
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}

// LSTM gates from PRE-SCALED pre-activations: lstm_pack_weights folds -log2(e) (sigmoid
// gates) and 2 log2(e) (the tanh gate) into the forward's bf16 weights Wp, so each gate is
// one v_exp_f32 (2^x) + add + v_rcp_f32 with no scaling multiply (the persistent forward's
// MFMA loop is vector-issue bound: cell math shares the SIMD's issue slots with the MFMAs)
constexpr float kLstmSigScale = -1.4426950408889634f;  // -log2(e)
constexpr float kLstmTanhScale = 2.8853900817779268f;  // 2 log2(e)
__device__ __forceinline__ float sigmoid_pre(float zs) { return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(zs)); }
__device__ __forceinline__ float tanh_pre(float zs) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(zs) + 1.0f);
}

__device__ __forceinline__ float tanhf_(float x) {
  // tanh(x) = 1 - 2/(exp(2x)+1); saturates cleanly for |x| large (exp -> inf or 0).
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * x) + 1.0f);
}

// Counter-based uniform in [0,1) (splitmix64 finaliser). Dropout masks are regenerated
// from (seed, flat index) in the backward pass instead of being stored; the same
// function is mirrored in wellflow/ops/reference.py for CPU tests.
__device__ __forceinline__ float uniform_hash(unsigned long long seed, unsigned long long idx) {
  unsigned long long z = seed + idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x < NT / 64) s = red[threadIdx.x];
  if (wid == 0) s = wave_sum(s);
  __syncthreads();
  return s;  // valid in wave 0 lanes
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD
// swizzle must be bijective"): blocks b, b+8, b+16... are dealt to the same XCD, so give
// each XCD a contiguous run of logical tiles so neighbouring tiles share its L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  constexpr int NX = 8;
  if (nwg < NX) return orig;
  const int q = nwg / NX, r = nwg % NX;
  const int x = orig % NX, i = orig / NX;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

}  // namespace wf
