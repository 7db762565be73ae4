// wellflow — instantiations of the persistent LSTM backward (lstm_persistent_bwd.inc.h), one
// object per (KT, NRT) variant (the build compiles this file once per variant line below).
// wf-build-variants: -DWF_KT=4 -DWF_NRT=4 | -DWF_KT=4 -DWF_NRT=8 | -DWF_KT=4 -DWF_NRT=16
// wf-build-variants: -DWF_KT=8 -DWF_NRT=4 | -DWF_KT=8 -DWF_NRT=8 | -DWF_KT=8 -DWF_NRT=16
// wf-build-variants: -DWF_KT=16 -DWF_NRT=4 | -DWF_KT=16 -DWF_NRT=8 | -DWF_KT=16 -DWF_NRT=16
#include "lstm_persistent_bwd.inc.h"

#define WF_PB_NAME2(a, b) launch_pb_##a##_##b
#define WF_PB_NAME(a, b) WF_PB_NAME2(a, b)

namespace wf {
int WF_PB_NAME(WF_KT, WF_NRT)(const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S, bf16_t* DG, const float* dcarry,
                              unsigned* sync, unsigned* stat, int grid, LstmDims d, hipStream_t s) {
  return launch_pb<WF_KT, WF_NRT>(WhhT, Cst, S, DG, dcarry, sync, stat, grid, d, s);
}
}  // namespace wf
