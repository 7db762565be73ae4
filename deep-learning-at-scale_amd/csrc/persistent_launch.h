// wellflow — host-side launch of the persistent (all-timesteps-in-one-launch) LSTM kernels.
//
// Every workgroup of a persistent grid must be resident at once (they wait on each other's
// per-step hand-offs). The launch checks that on the host — one 256-thread workgroup per CU
// and grid <= CUs x the occupancy query — and then uses a PLAIN launch by default:
//  * a plain launch of a grid that passes this check has the same residency as a cooperative
//    one (MI355X_MICROARCH.md "Residency and cooperative launch"), and skips the +15-20 us the
//    cooperative path costs per launch (price list row coop-launch), twice per training step;
//  * rocprofv3 7.2 (rocprofiler-sdk) dies with SIGSEGV inside its exit handlers after it has
//    traced a cooperative dispatch (profiles/r2_profiler_crash.md): with plain launches the
//    profiled binary is the production binary.
// WELLFLOW_COOP=1 selects hipLaunchCooperativeKernel (its own residency check) instead.
//
// Result: 1 = launched, 0 = this grid cannot be co-resident on this device (the caller falls
// back to per-step kernels), < 0 = -(hipError_t) of a failed launch (the caller raises).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

namespace wf {

inline bool persistent_coop_launch() {
  static const bool coop = [] {
    const char* v = std::getenv("WELLFLOW_COOP");
    return v != nullptr && v[0] == '1';
  }();
  return coop;
}

inline int persistent_launch(const void* f, int grid, void** args, hipStream_t s) {
  int per_cu = 0, dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -(int)hipErrorInvalidDevice;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 256, 0) != hipSuccess) return -(int)hipErrorInvalidValue;
  if (per_cu < 1 || grid > cus * per_cu) return 0;
  (void)hipGetLastError();  // a stale error from elsewhere must not be reported as ours
  const hipError_t e = persistent_coop_launch()
                           ? hipLaunchCooperativeKernel(f, dim3(grid), dim3(256), args, 0u, s)
                           : hipLaunchKernel(f, dim3(grid), dim3(256), args, 0u, s);
  return e == hipSuccess ? 1 : -(int)e;
}

}  // namespace wf
