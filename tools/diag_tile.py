"""Diagnostic: first layer where the bf16 LDS-DMA row-GEMM tile changes a forward result
(y, BN mean/invstd) -- tile A vs tile B, mod.py UNet(128, depth) bf16, one forward."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "thyroid-nodule-image-segmentation-unet-ddti_amd"),
                os.path.join(REPO, "tests")]
import torch  # noqa: E402

import unet_hip  # noqa: E402
from _helpers import inputs, options  # noqa: E402
from oracle import mod_ref_cpu as MO  # noqa: E402

DEV = torch.device("cuda:0")
ta, tb = int(sys.argv[1]), int(sys.argv[2])
depth, side = int(sys.argv[3]), int(sys.argv[4])
x, t = inputs(23, 2, side, side)
P = MO.make_params(9, 128, depth)
res = []
for tile in (ta, tb):
    m = unet_hip.ModUNet(1, 1, base_filters=128, depth=depth, mfma_dtype="bf16")
    sd = m.state_dict()
    sd.update({k: v.clone() for k, v in P.items()})
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    st = m.flatten_()
    with options(st.rt, rg16_tile=tile):
        with torch.no_grad():
            lg, ws = st.rt.forward(st.param_arena, st.bn_arena, st.nbt_arena, x.to(DEV), True)
        torch.cuda.synchronize()
    r = {"logits": lg.clone()}
    for i in range(2 * (2 * depth + 1)):
        v, off = st.rt.debug_view(ws, 2, side, side, True, 0, i)
        r[f"y{i}"] = v.clone()
        for kind, nm in ((3, "mean"), (4, "invstd")):
            r[f"{nm}{i}"] = st.rt.debug_view(ws, 2, side, side, True, kind, i).clone()
    res.append(r)
for k in res[0]:
    a, b = res[0][k], res[1][k]
    if not torch.equal(a, b):
        d = (a - b).abs()
        print(f"{k}: {int((a != b).sum())} differ, max {float(d.max()):.3e}")
print("done")
