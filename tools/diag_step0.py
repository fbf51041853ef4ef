"""Diagnostic: backward intermediates (d concat per level) and grads vs an fp64 oracle run,
with the fp64 dlogits fed straight into unet_backward (isolates the backward kernels)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "thyroid-nodule-image-segmentation-unet-ddti_amd"),
                os.path.join(REPO, "tests")]
import torch  # noqa: E402

from _helpers import hip_model, inputs  # noqa: E402
from oracle import unet_ref_cpu as O  # noqa: E402

torch.set_num_threads(16)
DEV = torch.device("cuda:0")
B, S = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (2, 64)
P32 = O.make_params(42)
x, t = inputs(1, B, S, S)
P = {k: v.double().requires_grad_() for k, v in P32.items()}
Bf = {k: (v.double() if v.is_floating_point() else v) for k, v in O.init_buffers().items()}
cats = []
_cat = torch.cat


def cat(ts, dim=0):
    o = _cat(ts, dim)
    o.retain_grad()
    cats.append(o)
    return o


torch.cat = cat
logits = O.forward(x.double(), P, Bf)
torch.cat = _cat
logits.retain_grad()
loss = O.bce_with_logits(logits, t.double()) + O.dice_loss(logits, t.double())
loss.backward()
dl = logits.grad.float()

m = hip_model(P32, DEV)
st = m.flatten_()
with torch.no_grad():
    lg, ws = st.rt.forward(st.param_arena, st.bn_arena, st.nbt_arena, x.to(DEV), training=True)
    grads = torch.zeros_like(st.param_arena)
    st.rt.backward(st.param_arena, dl.to(DEV).contiguous(), grads, ws)
torch.cuda.synchronize()


def nr(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


# cats[0] is CAT_3 (deepest), cats[3] is CAT_0
for lvl in range(4):
    ref = cats[3 - lvl].grad.permute(0, 2, 3, 1).reshape(-1, 2 * (64 << lvl))
    v, _ = st.rt.debug_view(ws, B, S, S, True, 7, lvl)
    got = v.cpu()
    C = 64 << lvl
    print(f"dcat[{lvl}] up {nr(got[:, :C], ref[:, :C]):.2e} skip {nr(got[:, C:], ref[:, C:]):.2e}")
off = 0
for name, p in P.items():
    n = p.numel()
    g = grads[off:off + n].cpu().view_as(p)
    off += n
    print(f"{name:28s} {nr(g, p.grad):.2e}")
