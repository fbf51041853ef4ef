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


def check_eval(m, forward_fn, x, t, tol=1e-4):
    """Resync the oracle from m's parameters AND running buffers and compare eval-mode
    (running-stat BN) logits at the north-star bar, the test masks (utils/trainer.py:217
    sigmoid > 0.5, bit-exact outside the forward error band) and the confusion counts of
    unet_mask_counts vs the reference's counting (utils/trainer.py:219-242: targets
    astype(uint8), TP/FP/FN/TN over every pixel).  Returns the near-boundary mask flips."""
    dev = next(m.parameters()).device
    Pc = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
    Bc = {k: v.detach().cpu().clone() for k, v in m.named_buffers()}
    m.eval()
    with torch.no_grad():
        lg = m(x.to(dev))
        ref = forward_fn(x, Pc, Bc, False)
    m.train()
    rl = ref.numpy()
    e = rel_max(lg.cpu().numpy(), rl)
    assert e <= tol, f"eval logits {e:.2e}"
    rt = m.flatten_().rt
    counts = torch.zeros(6, dtype=torch.int64, device=dev)
    mask = torch.empty(lg.shape, dtype=torch.uint8, device=dev)
    rt.mask_counts(lg, t.to(dev), counts, mask)
    ref_mask = O.mask_readout(ref).numpy()
    ok, nd = masks_agree(mask.cpu().numpy(), ref_mask, rl, 10 * tol * np.abs(rl).max())
    assert ok, f"{nd} eval mask bits differ away from the decision boundary"
    tg = t.numpy().astype(np.uint8)
    pr = mask.cpu().numpy().astype(bool)
    want = [int((pr & (tg == 1)).sum()), int((pr & (tg == 0)).sum()),
            int((~pr & (tg == 1)).sum()), int((~pr & (tg == 0)).sum())]
    assert counts.cpu().tolist()[:4] == want
    rp = ref_mask.astype(bool)  # vs the oracle's masks: only near-boundary pixels move
    ref_counts = [int((rp & (tg == 1)).sum()), int((rp & (tg == 0)).sum()),
                  int((~rp & (tg == 1)).sum()), int((~rp & (tg == 0)).sum())]
    assert sum(abs(a - b) for a, b in zip(want, ref_counts)) <= 2 * nd
    return nd


class options:
    """Set native kernel-schedule options (unet_set_option) for a block, restoring the
    previous values after it: runtimes are cached per device and network configuration."""

    def __init__(self, rt, **kv):
        self.rt, self.kv, self.old = rt, kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = self.rt.get_option(k)
            self.rt.set_option(k, v)
        return self.rt

    def __exit__(self, *exc):
        for k, v in self.old.items():
            self.rt.set_option(k, v)
        return False


def _to64(d):
    return {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in d.items()}


def _copy(d):
    return {k: v.clone() for k, v in d.items()}


def strict_resync_steps(m, train_step_fn, x, t, steps=3, lr=1e-4, floor0=5e-3, floor=1e-2):
    """Per-step parity with the oracle restarted from THIS path's state before every step
    (tests/test_gpu_parity.py::test_train_steps_strict_resync, generalised to any network
    through train_step_fn(P, B, opt, x, t) -> dict(logits, loss, grads)).

    Each step: the oracle takes this path's parameters, BN running statistics and Adam
    moments; logits must match it at the north-star bar (1e-4 of max|ref|), the loss at
    1e-5; every gradient is judged against the fp64 evaluation of the same graph, within 2x
    the largest fp32 oracle deviation from fp64 over nine fp32 noise realisations (x scaled
    by 1, 1 +- 1e-7 .. 1 +- 5e-7: each moves a different few ReLU inputs across
    zero; measured on mod.py UNet(64, 3) at step 0 they span 3e-5 .. 9e-3 on the small BN /
    ConvT bias gradients) and at least `floor0` (step 0) / `floor` (later steps, where
    the flips compound).  Returns the per-step worst gradient errors."""
    import unet_hip
    from oracle import unet_ref_cpu as O
    dev = next(m.parameters()).device
    opt = unet_hip.HipAdamW(m.parameters(), lr=lr)
    xd, td = x.to(dev), t.to(dev)
    worst = []
    for s in range(steps):
        Pc = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
        Bc = {k: v.detach().cpu().clone() for k, v in m.named_buffers()}
        r64 = train_step_fn(_to64(Pc), _to64(Bc), None, x.double(), t.double())
        spread = 0.0
        for eps in (1e-7, -1e-7, 2e-7, -2e-7, 3e-7, -3e-7, 5e-7, -5e-7):
            r32p = train_step_fn(_copy(Pc), _copy(Bc), None, x * (1 + eps), t)
            spread = max(spread, max(norm_rel(g, r64["grads"][k]) for k, g in r32p["grads"].items()))
        ref_opt = O.AdamWState(_copy(Pc), lr=lr)
        if s:
            for k, p in m.named_parameters():
                ref_opt.m[k] = opt.state[p]["exp_avg"].detach().cpu().clone()
                ref_opt.v[k] = opt.state[p]["exp_avg_sq"].detach().cpu().clone()
        ref_opt.step_count = s
        ref = train_step_fn(_copy(Pc), _copy(Bc), ref_opt, x, t)
        opt.zero_grad()
        logits = m(xd)
        losses = unet_hip.seg_losses(logits, td)
        loss = losses[0] + losses[1]
        loss.backward()
        e_l = rel_max(logits.detach().cpu().numpy(), ref["logits"].numpy())
        assert e_l <= 1e-4, f"step {s}: logits {e_l:.2e}"
        assert abs(loss.item() - ref["loss"].item()) <= 1e-5, f"step {s}: loss"
        e_hip = grad_errors(m, r64["grads"])
        e32d = {k: norm_rel(g, r64["grads"][k]) for k, g in ref["grads"].items()}
        e32 = max(e32d.values())
        e32p = max(e32, spread)
        env = max(2 * e32p, floor0 if s == 0 else floor)
        k_w = max(e_hip, key=e_hip.get)
        med = float(np.median(list(e_hip.values())))
        med32 = float(np.median(list(e32d.values())))
        print(f"step {s}: logits {e_l:.2e}; worst grad {k_w} {e_hip[k_w]:.2e} (fp32 oracle "
              f"{e32:.2e} / {e32p:.2e}, envelope {env:.2e}); median tensor {med:.2e} "
              f"(fp32 oracle {med32:.2e})")
        assert e_hip[k_w] <= env, f"step {s} {k_w}: hip {e_hip[k_w]:.2e}, envelope {env:.2e}"
        worst.append(e_hip[k_w])
        opt.step()
    return worst
