// Micro-benchmark: cycles per "slot" = one v_mfma_f32_16x16x32_bf16 + a VALU filler, one wave
// per SIMD (the persistent LSTM kernels' regime). Answers what the forward's fused micro-stage
// schedule can expect from the hardware: is a transcendental really free beside a 16x16x32
// MFMA, and what does a dependency chain of distance d between fillers cost?
//
//   hipcc --offload-arch=gfx950 -O3 tools/slot_bench.hip -o /tmp/slot_bench && /tmp/slot_bench
//
// Each variant runs 256 workgroups x 256 threads (one wave per SIMD on every CU) over 2048
// slots; s_memtime (shader clock) around the loop; reports the median over waves of
// cycles per slot.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define MF(acc) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b))

template <int V>
__global__ __launch_bounds__(256, 1) void slots(float* out, unsigned long long* cyc, float seed) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (short)(threadIdx.x + i);
    b[i] = (short)(threadIdx.x * 3 + i);
  }
  f32x4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = seed * (threadIdx.x + i) * 1e-3f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 256; ++it) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (s % 4 == 0) MF(acc0);
      if (s % 4 == 1) MF(acc1);
      if (s % 4 == 2) MF(acc2);
      if (s % 4 == 3) MF(acc3);
      if constexpr (V == 1) {  // independent v_exp per slot (8 chains, distance 8)
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[s]));
      } else if constexpr (V == 2) {  // v_exp chain of distance 2 (two chains alternating)
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[s & 1]));
      } else if constexpr (V == 3) {  // distance 1 (one chain)
        asm volatile("v_exp_f32 %0, %0" : "+v"(x[0]));
      } else if constexpr (V == 4) {  // two independent v_add
        asm volatile("v_add_f32 %0, 1.0, %0\n\tv_add_f32 %1, 1.0, %1" : "+v"(x[s]), "+v"(x[(s + 4) & 7]));
      } else if constexpr (V == 5) {  // exp -> add -> rcp chains (the gate pattern), distance 2
        const int k = s & 1;
        if ((s >> 1) % 3 == 0) asm volatile("v_exp_f32 %0, %0" : "+v"(x[k]));
        if ((s >> 1) % 3 == 1) asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(x[k]));
        if ((s >> 1) % 3 == 2) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[k]));
      } else if constexpr (V == 6) {  // same, distance 4 (four chains)
        const int k = s & 3;
        if ((s >> 2) % 2 == 0) asm volatile("v_exp_f32 %0, %0" : "+v"(x[k]));
        else asm volatile("v_rcp_f32 %0, %0" : "+v"(x[k]));
      } else if constexpr (V == 7) {  // v_exp + v_accvgpr_read of a different accumulator
        float r;
        asm volatile("v_exp_f32 %0, %0\n\tv_accvgpr_read_b32 %1, %2" : "+v"(x[s]), "=v"(r) : "a"(s < 4 ? acc2[0] : acc0[0]));
        x[(s + 1) & 7] += r * 1e-30f;
      } else if constexpr (V == 8) {  // fused form: MFMA and the exp in one asm statement
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
  float s = acc0[0] + acc1[1] + acc2[2] + acc3[3];
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// The forward's k-tile as it stands: 8 MFMAs per k-tile = 2 A fragments (VGPR, read from LDS
// one k-tile ahead with a counted lgkmcnt(2)) x 4 weight fragments (B, AGPR or VGPR), 8
// accumulators in AGPRs, a filler per MFMA (W: 0 none, 1 independent v_exp, 2 exp/rcp chains
// at distance 2 as in the micro-stages). KT k-tiles per "chunk", repeated.
template <int W, bool BAGPR, bool LDSA>
__global__ __launch_bounds__(256, 1) void ktile(float* out, unsigned long long* cyc, float seed) {
  constexpr int KT = 18;
  __shared__ __attribute__((aligned(16))) char smem[KT * 2 * 1024];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < KT * 2 * 1024 / 4; i += 256) reinterpret_cast<int*>(smem)[i] = i * 7;
  __syncthreads();
  bf16x8 w[4];
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 8; ++i) w[j][i] = (short)(threadIdx.x * (j + 1) + i);
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0, 0, 0, 0};
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = seed * (threadIdx.x + i) * 1e-3f;
  const unsigned base = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem) + lane * 16;
  bf16x8 a[2][2];
  for (int i = 0; i < 2; ++i)
    for (int k = 0; k < 8; ++k) a[0][i][k] = a[1][i][k] = (short)(lane + k + i);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 32; ++it) {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      if constexpr (LDSA) {
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[(kt + 1) & 1][0]) : "v"(base), "i"(((kt + 1) % KT) * 2048) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a[(kt + 1) & 1][1]) : "v"(base), "i"(((kt + 1) % KT) * 2048 + 1024) : "memory");
        asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(a[kt & 1][0]), "+v"(a[kt & 1][1])::"memory");
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int i = m >> 2, j = m & 3;
        if constexpr (BAGPR)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[m]) : "v"(a[kt & 1][i]), "a"(w[j]));
        else
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[m]) : "v"(a[kt & 1][i]), "v"(w[j]));
        if constexpr (W == 1) asm volatile("v_exp_f32 %0, %0" : "+v"(x[m]));
        if constexpr (W == 2) {
          if ((m >> 1) & 1) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[m & 1]));
          else asm volatile("v_exp_f32 %0, %0" : "+v"(x[m & 1]));
        }
      }
      asm volatile("" ::"v"(a[kt & 1][0]), "v"(a[kt & 1][1]));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int W, bool BAGPR, bool LDSA>
static void run_kt(const char* name) {
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 256 * 256 * 4);
  (void)hipMalloc(&cyc, 1024 * 8);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((ktile<W, BAGPR, LDSA>), dim3(256), dim3(256), 0, 0, out, cyc, 0.5f);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(1024);
  (void)hipMemcpy(h.data(), cyc, 1024 * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-58s %6.1f cycles/slot (median over waves; p10 %.1f p90 %.1f)\n", name, h[512] / (32.0 * 18 * 8),
         h[102] / (32.0 * 18 * 8), h[921] / (32.0 * 18 * 8));
  (void)hipFree(out);
  (void)hipFree(cyc);
}

template <int V>
static void run(const char* name) {
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 256 * 256 * 4);
  (void)hipMalloc(&cyc, 1024 * 8);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(slots<V>, dim3(256), dim3(256), 0, 0, out, cyc, 0.5f);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(1024);
  (void)hipMemcpy(h.data(), cyc, 1024 * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-58s %6.1f cycles/slot (median over waves; p10 %.1f p90 %.1f)\n", name, h[512] / 2048.0, h[102] / 2048.0,
         h[921] / 2048.0);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  run<0>("MFMA 16x16x32 only");
  run<1>("+ independent v_exp");
  run<2>("+ v_exp chain, distance 2 slots");
  run<3>("+ v_exp chain, distance 1 slot");
  run<4>("+ two independent v_add");
  run<5>("+ exp/add/rcp chains, distance 2");
  run<6>("+ exp/rcp chains, distance 4");
  run<7>("+ v_exp + v_accvgpr_read");
  run_kt<0, false, false>("k-tile: 8 acc, B VGPR, A fixed");
  run_kt<0, true, false>("k-tile: 8 acc, B AGPR, A fixed");
  run_kt<0, true, true>("k-tile: B AGPR, A from LDS (lgkmcnt 2)");
  run_kt<1, true, true>("k-tile: B AGPR, A from LDS, + v_exp");
  run_kt<2, true, true>("k-tile: B AGPR, A from LDS, + exp/rcp chains d=2");
  run_kt<2, false, true>("k-tile: B VGPR, A from LDS, + exp/rcp chains d=2");
  return 0;
}
