"""Debug: which option settings give non-finite gradients in one x3 training step (B=2, 128^2).
Prints, per setting, the non-finite counts of the logits and of every parameter gradient."""
import sys
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
sys.path.insert(0, "thyroid-nodule-image-segmentation-unet-ddti_amd")
from _helpers import hip_model, inputs, options  # noqa: E402
from oracle import unet_ref_cpu as O  # noqa: E402
import unet_hip  # noqa: E402

DEV = torch.device("cuda:0")
x, t = inputs(13, 2, 128, 128)
settings = [dict(x3_tile=-1, x3_n64=2, x3_r3=0), dict(x3_tile=0, x3_n64=2, x3_r3=0),
            dict(x3_tile=0, x3_n64=2, x3_r3=0, x3_1tap16=0), dict(x3_tile=1, x3_n64=2, x3_r3=0),
            dict(x3_tile=0, x3_n64=2, x3_r3=0, x3_wsched=0)]
for st in settings:
    m = hip_model(O.make_params(42), DEV)
    with options(m.flatten_().rt, **st):
        logits = m(x.to(DEV))
        l = unet_hip.seg_losses(logits, t.to(DEV))
        (l[0] + l[1]).backward()
        torch.cuda.synchronize()
    bad = {k: int((~torch.isfinite(p.grad)).sum()) for k, p in m.named_parameters() if p.grad is not None}
    bad = {k: v for k, v in bad.items() if v}
    print(st, "logits nonfinite", int((~torch.isfinite(logits)).sum()), "grads:", bad, flush=True)
    del m
