"""Shared test helpers (GPU parity against the CPU oracle)."""
import numpy as np
import torch

from oracle import unet_ref_cpu as O
from oracle import weights as Wt


def hip_model(P, dev, buffers=None):
    import unet_hip
    m = unet_hip.UNet(1, 1)
    sd = m.state_dict()
    for k, v in P.items():
        sd[k] = v.clone()
    for k, v in (buffers or O.init_buffers()).items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    return m.to(dev).train()


def rel_max(a, ref):
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(a - ref)) / max(np.max(np.abs(ref)), 1e-30))


def norm_rel(a, ref):
    a = torch.as_tensor(a).double()
    ref = torch.as_tensor(ref).double()
    return float((a - ref).norm() / max(float(ref.norm()), 1e-30))


def grad_errors(model, ref_grads):
    g = dict(model.named_parameters())
    return {k: norm_rel(g[k].grad.detach().cpu(), v) for k, v in ref_grads.items()}


def masks_agree(mask, ref_mask, ref_logits, tol):
    """Bit-exact masks except where the reference logit is within the forward error bound."""
    diff = mask != ref_mask
    if not diff.any():
        return True, 0
    near = np.abs(ref_logits) <= tol
    return bool(np.all(near[diff])), int(diff.sum())


def inputs(seed, B, H, W):
    return (torch.from_numpy(Wt.make_input(seed, B, 1, H, W)),
            torch.from_numpy(Wt.make_target(seed, B, H, W)))


def hip_mod_model(P, dev, base, depth, buffers=None):
    """models/mod.py UNet(base_filters=base, depth=depth) on the HIP path with params P."""
    import unet_hip
    from oracle import mod_ref_cpu as MO
    m = unet_hip.ModUNet(1, 1, base_filters=base, depth=depth)
    sd = m.state_dict()
    for k, v in P.items():
        sd[k] = v.clone()
    for k, v in (buffers or MO.init_buffers(base, depth)).items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    return m.to(dev).train()
