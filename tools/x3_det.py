"""GPU-box check: one training step (B=2, 256x256, model.py UNet) per schedule spec, each
spec run twice; reports bitwise equality of repeats and against the first spec, and the
norm-relative gap of the worst three gradient tensors.
usage: python tools/x3_det.py "" "x3_r3=0" "x3_wob=1 x3_r3=1" ..."""
import sys
sys.path[:0] = ["tests", ".", "thyroid-nodule-image-segmentation-unet-ddti_amd"]
import torch
import unet_hip
from _helpers import hip_model, inputs, norm_rel, options
from oracle import unet_ref_cpu as O

DEV = torch.device("cuda:0")
x, t = inputs(29, 2, 256, 256)
specs = sys.argv[1:] or ["", "x3_r3=0"]
res = []
for spec in specs:
    kv = dict((a, int(b)) for a, b in (o.split("=") for o in spec.split()))
    for rep in range(2):
        m = hip_model(O.make_params(42), DEV)
        with options(m.flatten_().rt, **kv):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        res.append((f"[{spec}]#{rep}", logits.detach().cpu().double(),
                    {k: p.grad.detach().cpu().double() for k, p in m.named_parameters()}))
        del m
base = res[0]
for r in res[1:]:
    same = torch.equal(r[1], base[1]) and all(torch.equal(r[2][k], base[2][k]) for k in r[2])
    gaps = sorted(((norm_rel(r[2][k], base[2][k]), k) for k in r[2]), reverse=True)[:3]
    print(f"{r[0]} vs {base[0]}: bitwise {same} logits {norm_rel(r[1], base[1]):.2e} "
          f"worst grads {[(f'{g:.1e}', k) for g, k in gaps]}", flush=True)
