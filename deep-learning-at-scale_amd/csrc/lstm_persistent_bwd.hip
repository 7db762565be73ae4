// wellflow — host launcher of the persistent LSTM backward (kernel: lstm_persistent_bwd.inc.h,
// instantiations: lstm_pb_parts.hip). SURVEY.md §2.4 K14.
#include <cstdlib>

#include "kernels.h"
#include "persistent_guard.h"
#include "persistent_launch.h"

namespace wf {

#define WF_PB_DECL(KT, NRT)                                                                              \
  int launch_pb_##KT##_##NRT(const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S, bf16_t* DG,          \
                             const float* dcarry, unsigned* sync, unsigned* stat, int grid, LstmDims d, \
                             hipStream_t s);
#define WF_PB_DECL_NRT(KT) WF_PB_DECL(KT, 4) WF_PB_DECL(KT, 8) WF_PB_DECL(KT, 16)
WF_PB_DECL_NRT(4)
WF_PB_DECL_NRT(8)
WF_PB_DECL_NRT(16)

namespace {
constexpr int PB_MAX_RT = 16;  // row tiles per workgroup (lstm_persistent_bwd.inc.h)

int launch_pb_variant(int KT, int NRT, const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S, bf16_t* DG,
                      const float* dcarry, unsigned* sync, unsigned* stat, int grid, LstmDims d, hipStream_t s) {
#define WF_PB_CASE(K)                                                                      \
  case K:                                                                                  \
    switch (NRT) {                                                                         \
      case 4: return launch_pb_##K##_4(WhhT, Cst, S, DG, dcarry, sync, stat, grid, d, s);   \
      case 8: return launch_pb_##K##_8(WhhT, Cst, S, DG, dcarry, sync, stat, grid, d, s);   \
      case 16: return launch_pb_##K##_16(WhhT, Cst, S, DG, dcarry, sync, stat, grid, d, s); \
      default: return 0;                                                                   \
    }
  switch (KT) {
    WF_PB_CASE(4)
    WF_PB_CASE(8)
    WF_PB_CASE(16)
    default: return 0;
  }
#undef WF_PB_CASE
}
}  // namespace

int persistent_split(int B, int row_quantum, int max_units, int cols, int cus, int* units_out,
                     unsigned unit_mask);  // lstm_persistent.hip

// Steps T-2 .. 0 of the backward in one launch per sub-batch (step T-1 must already be done:
// DG[T-1] and the dc carry written by lstm_bwd_last_kernel). 1 = launched, 0 = the shape /
// device cannot host the persistent schedule (nothing launched; the caller runs the per-step
// kernels), < 0 = -(hipError_t) of a failed launch.
int launch_lstm_bwd_persistent(const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S, bf16_t* DG,
                               const float* dcarry, unsigned* sync, long sync_words, LstmDims d,
                               hipStream_t s) {
  d.dbg &= kDbgMask;  // production: the test hook only (persistent_guard.h)
  if (d.T < 2) return 1;  // nothing after the last step
  const int G = 4 * d.H;
  if (d.H % 64 != 0 || d.B % 64 != 0) return 0;
  if (d.H != 128 && d.H != 256 && d.H != 512) return 0;
  if ((double)d.B * G * 2 >= 2147483647.0) return 0;  // 32-bit buffer offsets per step
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -(int)hipErrorInvalidDevice;
  const int NB = d.H / 64;
  // fewest sub-batches, then the fewest row tiles per workgroup (a multiple of 4: the row-tile
  // loop is unrolled by 4; at most PB_MAX_RT: the dc carry lives in registers), one WG per CU
  int u = 0;
  const int nsub = persistent_split(d.B, 64, PB_MAX_RT / 4, NB, cus, &u, 0xFu);
  if (nsub == 0) return 0;
  const int NRT = 4 * u, Bs = d.B / nsub, MB = Bs / (16 * NRT);
  if (sync_words < lstm_persistent_sync_total(MB)) return 0;
  unsigned* stat = sync + (sync_words - kPStatWords);  // running totals: never cleared here
  const int grid = MB * NB;
  // no per-launch reset: the hand-off words only count up (persistent_sync.h); the buffer is
  // zeroed at allocation and by NativeLSTM.reset_device_errors
  for (int k = 0; k < nsub; ++k) {
    LstmDims dk = d;
    dk.row_off = k * Bs;
    const int r = launch_pb_variant(d.H / 32, NRT, WhhT, Cst, S, DG, dcarry, sync, stat, grid, dk, s);
    if (r <= 0) return k == 0 ? r : (r < 0 ? r : -(int)hipErrorLaunchFailure);
  }
  return 1;
}

}  // namespace wf
