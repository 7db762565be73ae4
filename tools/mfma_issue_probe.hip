// Issue-cost probe for the persistent LSTM forward's MFMA loop (round 6 budget).
//
// Every CU runs one 256-thread workgroup (one wave per SIMD, like lstm_fwd_persistent_kernel);
// each wave repeats a "k-tile" of 8 v_mfma_f32_16x16x32_bf16 (2 A fragments x 4 B fragments,
// 8 independent accumulators) plus the fillers of the variant, and stamps s_memtime /
// s_memrealtime around the loop. Prints cycles per k-tile (shader clock) and the clock.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_issue_probe.hip -o /tmp/mfma_probe
//   ./mfma_probe            (all variants)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

constexpr int ITERS = 4096;

// V: 0 bare (B in AGPR) | 1 bare (B in VGPR) | 2 +1 v_exp per MFMA | 3 +2 v_add per MFMA
//    4 +2 ds_read_b128 + lgkmcnt(2) per k-tile | 5 = 2 + 4 | 6 = 5 + 1 LDS-DMA per 2 k-tiles
//    7 32x32x16: 4 MFMAs per k-tile (same FLOP), bare | 8 = 7 + 8 v_exp + 2 ds_read (8-VGPR B)
//    9 = 7 + 16 v_exp | 10 = 5 with v_exp then v_add per MFMA (the production stage mix)
template <int V>
__global__ __launch_bounds__(256, 1) void probe(const unsigned* __restrict__ src, unsigned long long* out,
                                                float* sink) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // random-ish operands (DVFS: zero data clocks higher)
  bf16x8 a[2], w[4];
  for (int i = 0; i < 2; ++i) {
    u32x4 v = *reinterpret_cast<const u32x4*>(src + ((blockIdx.x * 256 + threadIdx.x) * 8 + i * 4) % 65536);
    a[i] = __builtin_bit_cast(bf16x8, v);
  }
  for (int j = 0; j < 4; ++j) {
    u32x4 v = *reinterpret_cast<const u32x4*>(src + ((blockIdx.x * 77 + threadIdx.x * 3 + j * 4096) * 4) % 65536);
    w[j] = __builtin_bit_cast(bf16x8, v);
  }
  for (int i = threadIdx.x; i < 65536 / 16; i += 256)
    reinterpret_cast<u32x4*>(lds)[i] = *reinterpret_cast<const u32x4*>(src + (i * 4) % 65536);
  __syncthreads();
  f32x4 acc[8];
  f32x16 acc32[2];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < 2; ++i)
    for (int k = 0; k < 16; ++k) acc32[i][k] = 0.f;
  float e[16];
  for (int i = 0; i < 16; ++i) e[i] = (float)(lane + i) * 1e-3f;
  const unsigned rd = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)lds) + lane * 16 + wid * 4096;
  bf16x8 b0 = a[0], b1 = a[1];
  // the DMA variants' sources (the first 256 KiB of src) and the VGPR staging of V13 / V15
  const __amdgpu_buffer_rsrc_t vrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7FFFFFFF, 0x00020000);
  __amdgpu_buffer_rsrc_t srsrc = vrsrc;
  typedef unsigned u32x4b __attribute__((ext_vector_type(4)));
  u32x4b stg[4] = {};
  const unsigned* gsrc = src + lane * 4;  // 16 B per lane, 1 KiB per wave-instruction
  const unsigned wrl = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)lds) + 36864 + wid * 4096 + lane * 16;
  __builtin_amdgcn_s_barrier();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (V == 7 || V == 8 || V == 9) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if constexpr (V == 8) {
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %3, %4, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2"
                       : "+a"(acc32[m & 1]), "+v"(e[2 * m]), "+v"(e[2 * m + 1])
                       : "v"(a[m >> 1]), "a"(w[m]));
        } else if constexpr (V == 9) {
          asm volatile(
              "v_mfma_f32_32x32x16_bf16 %0, %5, %6, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_exp_f32 %3, "
              "%3\n\tv_exp_f32 %4, %4"
              : "+a"(acc32[m & 1]), "+v"(e[4 * m]), "+v"(e[4 * m + 1]), "+v"(e[4 * m + 2]), "+v"(e[4 * m + 3])
              : "v"(a[m >> 1]), "a"(w[m]));
        } else {
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc32[m & 1]) : "v"(a[m >> 1]), "a"(w[m]));
        }
      }
      if constexpr (V == 8) {
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(2)"
                     : "=v"(b0), "=v"(b1)
                     : "v"(rd)
                     : "memory");
        asm volatile("" ::"v"(b0), "v"(b1));
      }
    } else {
      if constexpr (V == 4 || V == 5 || V == 6 || V == 10 || V == 11 || V >= 12) {
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024\n\ts_waitcnt lgkmcnt(2)"
                     : "=v"(b0), "=v"(b1)
                     : "v"(rd)
                     : "memory");
        asm volatile("" ::"v"(b0), "v"(b1));
      }
      if constexpr (V == 12 || V == 14) {  // MUBUF LDS-DMA (4-B lane offsets), as the backward issues it
        constexpr int N = V == 12 ? 1 : 4;
        if (V == 14 || (it & 1))
#pragma unroll
          for (int q = 0; q < N; ++q)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(srsrc, (__attribute__((address_space(3))) void*)(lds + 32768 + wid * 4096 + q * 1024),
                                                     16, lane * 16, ((it & 255) * 1024 + q * 256) & 0x3FFFF, 0, 0);
      }
      if constexpr (V == 13 || V == 15) {  // the same bytes through VGPRs: buffer load, then ds_write_b128
        constexpr int N = V == 13 ? 1 : 4;
        if (V == 15 || (it & 1)) {
#pragma unroll
          for (int q = 0; q < N; ++q) {
            // issue cost only: the store writes an operand already in registers, the loads land
            // in a staging ring read once at the end (a real pipeline keeps them in flight)
            asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(wrl), "v"(b0), "i"(q * 1024) : "memory");
            // asm load: the compiler tracks nothing, so no wait is inserted for the in-flight
            // loads (their registers are rewritten in issue order; values unused until the end)
            // "+v": the staging registers stay allocated for the whole loop — with "=v" the
            // compiler reused an in-flight load's destination for a later ADDRESS register and
            // the late write-back faulted (illegal address, round 6)
            asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "+v"(stg[q]) : "v"(gsrc + (it & 63) * 256), "i"(q * 1024)
                         : "memory");
          }
        }
      }
      if constexpr (V == 6) {
        if (it & 1)
          __builtin_amdgcn_global_load_lds((const void*)(src + lane * 4 + (it & 255) * 256),
                                           (__attribute__((address_space(3))) void*)(lds + 32768 + wid * 1024), 16, 0,
                                           0);
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int i = m >> 2, j = m & 3;
        if constexpr (V == 1) {
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[m]) : "v"(a[i]), "v"(w[j]));
        } else if constexpr (V == 2 || V == 5 || V == 6 || V >= 12) {
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\tv_exp_f32 %1, %1"
                       : "+a"(acc[m]), "+v"(e[m])
                       : "v"(a[i]), "a"(w[j]));
        } else if constexpr (V == 11) {  // V10 with the accumulators in VGPRs
          if (m & 1)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %3, %4, %0\n\tv_add_f32 %1, 1.0, %1\n\tv_add_f32 %2, 1.0, %2"
                         : "+v"(acc[m]), "+v"(e[m]), "+v"(e[m + 8])
                         : "v"(a[i]), "a"(w[j]));
          else
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\tv_exp_f32 %1, %1"
                         : "+v"(acc[m]), "+v"(e[m])
                         : "v"(a[i]), "a"(w[j]));
        } else if constexpr (V == 10) {
          if (m & 1)
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %3, %4, %0\n\tv_add_f32 %1, 1.0, %1\n\tv_add_f32 %2, 1.0, %2"
                         : "+a"(acc[m]), "+v"(e[m]), "+v"(e[m + 8])
                         : "v"(a[i]), "a"(w[j]));
          else
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0\n\tv_exp_f32 %1, %1"
                         : "+a"(acc[m]), "+v"(e[m])
                         : "v"(a[i]), "a"(w[j]));
        } else if constexpr (V == 3) {
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %3, %4, %0\n\tv_add_f32 %1, 1.0, %1\n\tv_add_f32 %2, 1.0, %2"
                       : "+a"(acc[m]), "+v"(e[m]), "+v"(e[m + 8])
                       : "v"(a[i]), "a"(w[j]));
        } else {
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[m]) : "v"(a[i]), "a"(w[j]));
        }
      }
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
  for (int i = 0; i < 2; ++i) s += acc32[i][0] + acc32[i][15];
  for (int i = 0; i < 16; ++i) s += e[i];
  // the staging registers are operands of the wait: no read of them (and no reuse of their
  // registers) can move above it while the asm loads are in flight (round 6: a late write-back
  // into a register the compiler had reused for an address faulted)
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(stg[0]), "+v"(stg[1]), "+v"(stg[2]), "+v"(stg[3]) :: "memory");
  s += (float)b0[0] + (float)b1[7] + (float)(stg[0][0] + stg[1][1] + stg[2][2] + stg[3][3]);
  sink[blockIdx.x * 256 + threadIdx.x] = s;
  if (lane == 0) {
    out[(blockIdx.x * 4 + wid) * 2] = t1 - t0;
    out[(blockIdx.x * 4 + wid) * 2 + 1] = r1 - r0;
  }
}

template <int V>
void run(const char* name, unsigned* src, unsigned long long* out, float* sink, int grid) {
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe<V>, dim3(grid), dim3(256), 0, 0, src, out, sink);
  const hipError_t err = hipDeviceSynchronize();
  if (err != hipSuccess) {
    std::printf("%s: %s\n", name, hipGetErrorString(err));
    std::exit(1);
  }
  std::vector<unsigned long long> h(grid * 8);
  hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int i = 0; i < grid * 4; ++i) {
    cyc += (double)h[2 * i];
    rt += (double)h[2 * i + 1];
  }
  cyc /= grid * 4;
  rt /= grid * 4;
  const double per = cyc / ITERS;
  const double ghz = cyc / (rt * 10.0);  // s_memrealtime: 100 MHz
  std::printf("%-44s %7.1f cyc/k-tile  %5.2f cyc/MFMA-16  clock %.2f GHz  %.3f us/k-tile\n", name, per,
              per / 8.0, ghz, rt * 10.0 / 1000.0 / ITERS);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  unsigned *src;
  unsigned long long* out;
  float* sink;
  hipMalloc(&src, 65536 * 4 * 2);
  hipMalloc(&out, (size_t)cus * 8 * 8);
  hipMalloc(&sink, (size_t)cus * 256 * 4);
  std::vector<unsigned> h(65536 * 2);
  unsigned x = 12345;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (x & 0x3FFF3FFFu) | 0x3C003C00u;  // finite bf16 pairs in ~[1, 4)
  }
  hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  std::printf("grid %d workgroups x 256 threads (1 wave per SIMD), %d k-tiles per wave\n", cus, ITERS);
  run<0>("0 8x16x16x32, B in AGPR", src, out, sink, cus);
  run<1>("1 8x16x16x32, B in VGPR", src, out, sink, cus);
  run<2>("2 + v_exp per MFMA", src, out, sink, cus);
  run<3>("3 + 2 v_add per MFMA", src, out, sink, cus);
  run<4>("4 + 2 ds_read_b128 + lgkmcnt(2)", src, out, sink, cus);
  run<5>("5 + v_exp + ds_reads", src, out, sink, cus);
  run<10>("10 + exp/2add alternating + ds_reads", src, out, sink, cus);
  run<11>("11 = 10 with VGPR accumulators", src, out, sink, cus);
  run<6>("6 = 5 + LDS-DMA per 2 k-tiles", src, out, sink, cus);
  run<12>("12 = 5 + MUBUF LDS-DMA per 2 k-tiles", src, out, sink, cus);
  run<14>("14 = 5 + 4 MUBUF LDS-DMA per k-tile", src, out, sink, cus);
  // 13 / 15 (loads through VGPRs + ds_write_b128) are not run: their asm loads are only safe
  // while the compiler keeps every staging register allocated (see the wait above)
  run<7>("7 4x32x32x16 bare", src, out, sink, cus);
  run<8>("8 32x32: + 2 v_exp per MFMA + ds_reads", src, out, sink, cus);
  run<9>("9 32x32: + 4 v_exp per MFMA", src, out, sink, cus);
  hipFree(src);
  hipFree(out);
  hipFree(sink);
  return 0;
}
