"""GPU-box check: one bf16 training step of BASELINE config 4's network (models/mod.py
UNet base 128, depth 5) at 1 x 256 x 256 per schedule spec; reports bitwise equality with
the first spec.  usage: python tools/c4_det.py "" "rg16_ob=1" ..."""
import sys
sys.path[:0] = ["tests", ".", "thyroid-nodule-image-segmentation-unet-ddti_amd"]
import torch
import unet_hip
from _helpers import inputs, norm_rel, options
from oracle import mod_ref_cpu as MO

DEV = torch.device("cuda:0")
x, t = inputs(37, 2, 256, 256)
P = MO.make_params(41, 128, 5)
res = []
for spec in sys.argv[1:] or [""]:
    kv = dict((a, int(b)) for a, b in (o.split("=") for o in spec.split()))
    m = unet_hip.ModUNet(1, 1, base_filters=128, depth=5, mfma_dtype="bf16")
    sd = m.state_dict()
    for k, v in P.items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    with options(m.flatten_().rt, **kv):
        logits = m(x.to(DEV))
        l = unet_hip.seg_losses(logits, t.to(DEV))
        (l[0] + l[1]).backward()
        torch.cuda.synchronize()
    res.append((f"[{spec}]", logits.detach().cpu().double(),
                {k: p.grad.detach().cpu().double() for k, p in m.named_parameters()}))
    del m
base = res[0]
for r in res[1:]:
    same = torch.equal(r[1], base[1]) and all(torch.equal(r[2][k], base[2][k]) for k in r[2])
    gaps = sorted(((norm_rel(r[2][k], base[2][k]), k) for k in r[2]), reverse=True)[:3]
    print(f"{r[0]} vs {base[0]}: bitwise {same} logits {norm_rel(r[1], base[1]):.2e} "
          f"worst grads {[(f'{g:.1e}', k) for g, k in gaps]}", flush=True)
