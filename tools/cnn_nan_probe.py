"""Where does the fused CNN backward produce non-finite gradients? (round-5 debug probe)
Runs the failing test's setup and reports the non-finite entries per gradient block and in the
backward partial buffers."""
import sys

import torch

sys.path.insert(0, ".")
from wellflow.models.cnn import CNN1DRegressor, NativeCNN  # noqa: E402

DEV = "cuda:0"
torch.manual_seed(1)
ref = CNN1DRegressor(dropout=0.0).init_keras(3).to(DEV)
for B, batch in ((40, 64), (64, 64), (4096, 4096)):
    eng = NativeCNN(ref.layout, batch=batch, device=DEV, dropout=0.0, loss="mae_clip")
    eng.params.copy_(ref.to_flat().to(DEV))
    eng.sync_weights()
    x, y = torch.randn(B, 48, 1, device=DEV), torch.randn(B, 12, device=DEV)
    eng.part_wd.fill_(7.0)
    eng.part_wc.fill_(7.0)
    eng.forward_backward(x, y, grad_scale=1.0 / (B * 12))
    torch.cuda.synchronize()
    gWc, gWd, gbd = eng.lay.views(eng.grads)
    print(f"B={B} batch={batch}")
    for nm, t in (("gWc", gWc), ("gWd", gWd), ("gbd", gbd), ("dout", eng.dout), ("part_wd", eng.part_wd),
                  ("part_wc", eng.part_wc), ("part_f", eng.part_f), ("WcA", eng.WcA.float()), ("WdB", eng.WdB.float()),
                  ("WdF", eng.WdF.float())):
        bad = (~torch.isfinite(t)).nonzero()
        print(f"  {nm:8s} shape {tuple(t.shape)} nonfinite {bad.shape[0]}", bad[:8].flatten().tolist())
