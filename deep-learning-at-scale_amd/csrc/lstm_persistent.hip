// wellflow — host launcher of the persistent LSTM forward (kernel: lstm_persistent_fwd.inc.h,
// instantiations: lstm_pf_parts.hip). SURVEY.md §2.4 K13.
#include <cstdlib>

#include "kernels.h"
#include "persistent_guard.h"
#include "persistent_launch.h"

namespace wf {

#define WF_PF_DECL(KT, NC)                                                                            \
  int launch_pf_##KT##_##NC(bf16_t* XH, const bf16_t* Wp, bf16_t* Cst, bf16_t* S, unsigned* sync, \
                            unsigned* stat, int grid, LstmDims d, hipStream_t s);
#define WF_PF_DECL_NC(KT) WF_PF_DECL(KT, 1) WF_PF_DECL(KT, 2) WF_PF_DECL(KT, 4) WF_PF_DECL(KT, 8)
WF_PF_DECL_NC(6)
WF_PF_DECL_NC(10)
WF_PF_DECL_NC(18)
WF_PF_DECL_NC(8)
WF_PF_DECL_NC(12)
WF_PF_DECL(20, 1)
WF_PF_DECL(20, 8)

namespace {
constexpr int PF_ROWS = 32;  // rows per ring chunk (lstm_persistent_fwd.inc.h)

int launch_pf_variant(int KT, int NC, bf16_t* XH, const bf16_t* Wp, bf16_t* Cst, bf16_t* S, unsigned* sync,
                      unsigned* stat, int grid, LstmDims d, hipStream_t s) {
#define WF_PF_CASE(K)                                                     \
  case K:                                                                 \
    switch (NC) {                                                         \
      case 1: return launch_pf_##K##_1(XH, Wp, Cst, S, sync, stat, grid, d, s); \
      case 2: return launch_pf_##K##_2(XH, Wp, Cst, S, sync, stat, grid, d, s); \
      case 4: return launch_pf_##K##_4(XH, Wp, Cst, S, sync, stat, grid, d, s); \
      case 8: return launch_pf_##K##_8(XH, Wp, Cst, S, sync, stat, grid, d, s); \
      default: return 0;                                                  \
    }
  switch (KT) {
    WF_PF_CASE(6)
    WF_PF_CASE(10)
    WF_PF_CASE(18)
    WF_PF_CASE(8)
    WF_PF_CASE(12)
    case 20:
      if (NC == 1) return launch_pf_20_1(XH, Wp, Cst, S, sync, stat, grid, d, s);
      if (NC == 8) return launch_pf_20_8(XH, Wp, Cst, S, sync, stat, grid, d, s);
      return 0;
    default: return 0;
  }
#undef WF_PF_CASE
}
}  // namespace

// sync buffer (uint32 words): one 64-B line of monotonic hand-off words per row block after a
// 16-word head (persistent_sync.h: launch epoch, group arrival counters, tagged error word;
// zeroed once, never by a launch) and the 64-word completion STAT block at the END
// (persistent_guard.h: sticky spin-timeout bit and running totals; NativeLSTM.check_device_errors
// reads it).
int lstm_persistent_sync_words(int row_blocks) { return 16 + 16 * row_blocks; }
int dbg_mask() { return kDbgMask; }
long lstm_persistent_sync_total(int row_blocks) { return lstm_persistent_sync_words(row_blocks) + kPStatWords; }

// Batch split for the persistent schedules: the fewest equal sub-batches (launched one after
// the other on the stream, each a full persistent launch over its row range, d.row_off) whose
// grid of `rows_per_unit * units` rows per workgroup fits one workgroup per CU. Returns the
// number of sub-batches (0 = none fits) and the chosen units per workgroup; bit log2(u) of
// unit_mask says the variant with u units per workgroup is built.
int persistent_split(int B, int row_quantum, int max_units, int cols, int cus, int* units_out, unsigned unit_mask) {
  for (int nsub = 1; nsub <= 64; ++nsub) {
    if (B % nsub != 0) continue;
    const int Bs = B / nsub;
    if (Bs % row_quantum != 0) continue;
    for (int u = 1; u <= max_units; u *= 2) {
      if (((unit_mask >> __builtin_ctz((unsigned)u)) & 1u) == 0) continue;  // variant not built
      if (Bs % (row_quantum * u) == 0 && (Bs / (row_quantum * u)) * cols <= cus) {
        *units_out = u;
        return nsub;
      }
    }
  }
  return 0;
}

// 1 = launched, 0 = the shape or device cannot host the persistent schedule (nothing launched;
// the caller runs the per-step kernels), < 0 = -(hipError_t) of a failed launch.
// Batches larger than one co-resident grid run as consecutive sub-batch launches (no cap on B).
int launch_lstm_fwd_persistent(bf16_t* XH, const bf16_t* Wp, bf16_t* Cst, bf16_t* S, unsigned* sync,
                               long sync_words, LstmDims d, hipStream_t s) {
  d.dbg &= kDbgMask;  // production: the test hook only (persistent_guard.h)
  const int KA = d.KX + d.H, G = 4 * d.H;
  if ((double)d.B * KA * 2 >= 2147483647.0) return 0;  // 32-bit buffer offsets within one timestep slab
  if (d.KX % 64 != 0 || KA % 64 != 0 || G % 256 != 0 || d.B % PF_ROWS != 0) return 0;
  if (d.KX != 64 && d.KX != 128) return 0;  // F <= 127
  if (d.H != 128 && d.H != 256 && d.H != 512) return 0;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -(int)hipErrorInvalidDevice;
  const int NB = G / 256;
  // fewest sub-batches, then the fewest 32-row chunks per workgroup, one workgroup per CU
  int NC = 0;
  const int nsub = persistent_split(d.B, PF_ROWS, 8, NB, cus, &NC, KA / 32 == 20 ? 0x9u : 0xFu);
  if (nsub == 0) return 0;
  const int Bs = d.B / nsub, MB = Bs / (PF_ROWS * NC);
  if (sync_words < lstm_persistent_sync_total(MB)) return 0;
  unsigned* stat = sync + (sync_words - kPStatWords);  // running totals: never cleared here
  const int grid = MB * NB;
  // no per-launch reset: the hand-off words only count up (persistent_sync.h); the buffer is
  // zeroed at allocation and by NativeLSTM.reset_device_errors
  for (int k = 0; k < nsub; ++k) {
    LstmDims dk = d;
    dk.row_off = k * Bs;
    // KA / 32 = 6, 10, 18: H = 128, 256, 512
    const int r = launch_pf_variant(KA / 32, NC, XH, Wp, Cst, S, sync, stat, grid, dk, s);
    if (r <= 0) return k == 0 ? r : (r < 0 ? r : -(int)hipErrorLaunchFailure);
  }
  return 1;
}

}  // namespace wf
