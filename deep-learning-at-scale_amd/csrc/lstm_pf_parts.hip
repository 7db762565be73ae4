// wellflow — instantiations of the persistent LSTM forward (lstm_persistent_fwd.inc.h), one
// object per (KT, NC) variant: the build (_build.py) compiles this file once per line of the
// variant list below with those -D flags, so the slow unrolled instantiations compile in
// parallel and a kernel edit rebuilds in the time of the slowest one.
// wf-build-variants: -DWF_KT=6 -DWF_NC=1 | -DWF_KT=6 -DWF_NC=2 | -DWF_KT=6 -DWF_NC=4 | -DWF_KT=6 -DWF_NC=8
// wf-build-variants: -DWF_KT=10 -DWF_NC=1 | -DWF_KT=10 -DWF_NC=2 | -DWF_KT=10 -DWF_NC=4 | -DWF_KT=10 -DWF_NC=8
// wf-build-variants: -DWF_KT=18 -DWF_NC=1 | -DWF_KT=18 -DWF_NC=2 | -DWF_KT=18 -DWF_NC=4 | -DWF_KT=18 -DWF_NC=8
// KX = 128 (64 <= F <= 127): KT = 8 / 12 / 20 for H = 128 / 256 / 512
// wf-build-variants: -DWF_KT=8 -DWF_NC=1 | -DWF_KT=8 -DWF_NC=2 | -DWF_KT=8 -DWF_NC=4 | -DWF_KT=8 -DWF_NC=8
// wf-build-variants: -DWF_KT=12 -DWF_NC=1 | -DWF_KT=12 -DWF_NC=2 | -DWF_KT=12 -DWF_NC=4 | -DWF_KT=12 -DWF_NC=8
// (KT = 20 at NC = 2 / 4 spills hundreds of VGPRs: the launcher uses NC = 1 or 8 there)
// wf-build-variants: -DWF_KT=20 -DWF_NC=1 | -DWF_KT=20 -DWF_NC=8
#include "lstm_persistent_fwd.inc.h"

#define WF_PF_NAME2(a, b) launch_pf_##a##_##b
#define WF_PF_NAME(a, b) WF_PF_NAME2(a, b)

namespace wf {
int WF_PF_NAME(WF_KT, WF_NC)(bf16_t* XH, const bf16_t* Wp, bf16_t* Cst, bf16_t* S, unsigned* sync, unsigned* stat,
                             int grid, LstmDims d, hipStream_t s) {
  return launch_pf<WF_KT, WF_NC>(XH, Wp, Cst, S, sync, stat, grid, d, s);
}
}  // namespace wf
