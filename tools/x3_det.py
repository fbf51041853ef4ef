"""GPU-box check: is the x3 training step deterministic per schedule in a fresh process?
Runs x3_r3 = 1, 0, 1, 0 (and 2) on the same inputs and reports bitwise equality of repeats
and the norm-relative gradient gap between schedules (per tensor, worst three)."""
import sys
sys.path[:0] = ["tests", ".", "thyroid-nodule-image-segmentation-unet-ddti_amd"]
import torch
import unet_hip
from _helpers import hip_model, inputs, norm_rel, options
from oracle import unet_ref_cpu as O

DEV = torch.device("cuda:0")
x, t = inputs(29, 2, 256, 256)
res = []
for r3 in (1, 0, 1, 0, 2):
    m = hip_model(O.make_params(42), DEV)
    with options(m.flatten_().rt, x3_r3=r3):
        logits = m(x.to(DEV))
        l = unet_hip.seg_losses(logits, t.to(DEV))
        (l[0] + l[1]).backward()
        torch.cuda.synchronize()
    res.append((r3, logits.detach().cpu().double(),
                {k: p.grad.detach().cpu().double() for k, p in m.named_parameters()}))
    del m
for i in range(len(res)):
    for j in range(i):
        a, b = res[i], res[j]
        same = torch.equal(a[1], b[1]) and all(torch.equal(a[2][k], b[2][k]) for k in a[2])
        gaps = sorted(((norm_rel(a[2][k], b[2][k]), k) for k in a[2]), reverse=True)[:3]
        print(f"run{i}(r3={a[0]}) vs run{j}(r3={b[0]}): bitwise {same} logits {norm_rel(a[1], b[1]):.2e} "
              f"worst grads {[(f'{g:.1e}', k) for g, k in gaps]}", flush=True)
