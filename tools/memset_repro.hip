// Standalone repro for profiles/r3_early_exit.md: does a hipMemsetAsync node captured in a
// hipGraph zero its region on every replay, before and after hipHostMalloc? Args: word offset
// into a hipMalloc'd buffer, word count, replays. Prints per-replay nonzero words + word 0.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 2; } } while (0)
__global__ void poison(int* p, int n) { for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0x7f7f7f7f; }
__global__ void probe(const int* p, int n, int* out) {
  int bad = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) bad += p[i] != 0;
  atomicAdd(out, bad);
  if (threadIdx.x == 0) out[1] = p[0];
}
int main(int argc, char** argv) {
  const int off = argc > 1 ? atoi(argv[1]) : 1, n = argc > 2 ? atoi(argv[2]) : 527, reps = argc > 3 ? atoi(argv[3]) : 8;
  int *buf, *out, h[2], fails = 0;
  void* pinned = nullptr;
  CK(hipMalloc(&buf, 1 << 20));
  CK(hipMalloc(&out, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(poison, 1, 256, 0, s, buf, off + n + 16);
  CK(hipMemsetAsync(buf + off, 0, sizeof(int) * (size_t)n, s));
  CK(hipMemsetAsync(out, 0, 64, s));
  hipLaunchKernelGGL(probe, 1, 256, 0, s, buf + off, n, out);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int r = 0; r < 2 * reps; ++r) {
    if (r == reps) CK(hipHostMalloc(&pinned, 64 << 20, hipHostMallocDefault));  // as the job's eval slots
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h, out, 8, hipMemcpyDeviceToHost));
    fails += h[0] != 0;
    printf("off=%d B n=%d B replay %2d %s: nonzero words %d, word0 0x%08x\n", 4 * off, 4 * n, r,
           r >= reps ? "after hipHostMalloc " : "before hipHostMalloc", h[0], (unsigned)h[1]);
  }
  printf("RESULT off=%d B size=%d B: %d of %d replays left nonzero words\n", 4 * off, 4 * n, fails, 2 * reps);
  return fails ? 1 : 0;
}
