"""GPU parity of the HIP path (libunet_hip.so through its C ABI) against the CPU oracle and
the reference-generated golden fixtures.

Tolerances (north star / SURVEY.md §8c):
* forward logits: max|d| <= 1e-4 * max|ref|   ("1e-4 relative fp32")
* losses: |d| <= 1e-5 (absolute, losses are O(1))
* masks: bit-exact except where |ref logit| <= 1e-3 * max|ref| (forward error bound)
* gradients: norm-relative <= 1e-2 per tensor (the reference's own fp32-vs-fp64 error is
  ~4e-3); in practice the kernels land around 1e-5..1e-4
* AdamW-updated params: |d| <= 3e-7 absolute at lr 1e-5 (identical op order), except where
  the reference gradient is at fp32 noise level (Adam's first steps are ~lr*sign(g))
"""
import os

import numpy as np
import pytest
import torch

from _helpers import check_eval, grad_errors, hip_model, inputs, masks_agree, norm_rel, rel_max
from oracle import unet_ref_cpu as O
from oracle import weights as Wt

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
LOGIT_TOL = 1e-4
GRAD_TOL = 1e-2
FLIP_TOL = 5e-3  # gradient shift of a few ReLU-boundary flips (test_train_steps_strict_resync)


@pytest.fixture(autouse=True, scope="module")
def _threads():
    torch.set_num_threads(min(16, os.cpu_count() or 1))


def _golden(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def _step(m, opt, x, t, w_bce=1.0, w_dice=1.0):
    import unet_hip
    opt.zero_grad()
    logits = m(x)
    losses = unet_hip.seg_losses(logits, t)
    loss = w_bce * losses[0] + w_dice * losses[1]
    loss.backward()
    opt.step()
    return logits.detach(), losses.detach(), loss.detach()


def test_forward_layers_match_oracle():
    """Every conv layer's post-ReLU output (pre-BN) vs the oracle, train-mode BN, B=2 64x64."""
    P = O.make_params(42)
    x, _ = inputs(1, 2, 64, 64)
    rec = []
    ref = O.forward(x, P, O.init_buffers(), True, record=rec)
    m = hip_model(P, DEV)
    st = m.flatten_()
    with torch.no_grad():
        logits, ws = st.rt.forward(st.param_arena, st.bn_arena, st.nbt_arena, x.to(DEV), training=True)
    torch.cuda.synchronize()
    errs = []
    for i in range(18):
        v, off = st.rt.debug_view(ws, 2, 64, 64, True, 0, i)
        C = rec[i].shape[1]
        got = v[:, off:off + C].cpu().numpy()
        want = rec[i].permute(0, 2, 3, 1).reshape(-1, C).numpy()
        errs.append(rel_max(got, want))
    assert max(errs) <= LOGIT_TOL, f"per-layer rel errors: {np.array(errs)}"
    assert rel_max(logits.cpu().numpy(), ref.numpy()) <= LOGIT_TOL


def test_train_steps_match_golden(golden_dir):
    """Three full training steps (fwd, BCE+Dice, bwd, AdamW) vs the reference's own outputs.

    Step 0 is held to the strict bars.  Adam's first updates are ~lr*sign(g), so elements
    whose reference gradient is at fp32 noise level can move by 2*lr in either
    implementation; the trajectories then differ at ~1e-4 relative and steps 1-2 are
    compared to the golden trajectory at 2e-3 (logits) and their gradients at 10 % or twice
    the spread of the fp32 oracle's own trajectory under 1e-7-level input noise, whichever
    is larger -- and, strictly, to the oracle re-started from this path's own parameters
    (test_train_steps_strict_resync)."""
    import unet_hip
    f = _golden(golden_dir, "unet_b2_64.npz")
    m = hip_model(O.make_params(42), DEV)
    opt = unet_hip.HipAdamW(m.parameters(), lr=1e-5)
    x, t = torch.from_numpy(f["x"]).to(DEV), torch.from_numpy(f["t"]).to(DEV)
    spec = O.param_spec()
    tiny = None
    # steps 1-2: the fp32 reference trajectory itself moves under fp32 noise (inputs scaled
    # by 1 +- 1e-7 .. 1 +- 5e-7): Adam's sign-noise updates send a few small gradients away
    # (encoder4.0.bias at step 2: up to 18.7 % for x * (1 + 2e-7)).  The step >= 1 gradient
    # bars are max(10 %, 2x that spread).
    spread_n = np.zeros((3, len(spec)))
    spread_s = np.zeros((3, len(spec)))
    for eps in (1e-7, -1e-7, 2e-7, -2e-7, 3e-7, -3e-7, 5e-7, -5e-7):
        Pr, Br = O.make_params(42), O.init_buffers()
        opt_r = O.AdamWState(Pr, lr=1e-5)
        xr, tr = torch.from_numpy(f["x"]) * (1 + eps), torch.from_numpy(f["t"])
        for s in range(3):
            r = O.train_step(Pr, Br, opt_r, xr, tr)
            for ti, item in enumerate(spec):
                g = r["grads"][item[0]].double().reshape(-1)
                idx = np.floor(Wt.uniform(7, 3000 + ti, 64) * g.numel()).astype(np.int64)
                spread_n[s, ti] = max(spread_n[s, ti], abs(g.norm().item() - f[f"s{s}_grad_norm"][ti]))
                spread_s[s, ti] = max(spread_s[s, ti],
                                      float(np.max(np.abs(g[idx].numpy() - f[f"s{s}_grad_samp"][ti]))))
    for s in range(3):
        tol = LOGIT_TOL if s == 0 else 2e-3
        logits, losses, loss = _step(m, opt, x, t)
        ref = f[f"s{s}_logits"]
        lg = logits.cpu().numpy()
        assert rel_max(lg, ref) <= tol, f"step {s} logits"
        ok, nd = masks_agree((torch.sigmoid(logits) > 0.5).cpu().numpy().astype(np.uint8),
                             f[f"s{s}_mask"], ref, 10 * tol * np.abs(ref).max())
        assert ok, f"step {s}: {nd} mask bits differ away from the decision boundary"
        assert abs(losses[0].item() - float(f[f"s{s}_bce"])) <= (1e-5 if s == 0 else 1e-4)
        assert abs(losses[1].item() - float(f[f"s{s}_dice"])) <= (1e-5 if s == 0 else 1e-4)
        # gradients: per-tensor norm and the 64 fixed samples, relative to the tensor norm
        norms = f[f"s{s}_grad_norm"]
        samp = f[f"s{s}_grad_samp"]
        gtol = GRAD_TOL if s == 0 else 10 * GRAD_TOL  # trajectories drift after step 0
        for ti, item in enumerate(spec):
            g = dict(m.named_parameters())[item[0]].grad.detach().double().cpu().reshape(-1)
            idx = np.floor(Wt.uniform(7, 3000 + ti, 64) * g.numel()).astype(np.int64)
            bn = max(gtol * norms[ti], 2 * spread_n[s, ti]) if s else gtol * norms[ti]
            bs = max(gtol * norms[ti], 2 * spread_s[s, ti]) if s else gtol * norms[ti]
            assert abs(g.norm().item() - norms[ti]) <= bn, item[0]
            assert np.max(np.abs(g[idx].numpy() - samp[ti])) <= bs, item[0]
        # post-AdamW parameters: 2 ulp, except sign-noise elements (|g_ref| < 1% of rms)
        pnow = dict(m.named_parameters())
        ps = np.stack([pnow[it[0]].detach().cpu().reshape(-1)[torch.from_numpy(
            np.floor(Wt.uniform(7, 3000 + ti, 64) * pnow[it[0]].numel()).astype(np.int64))].numpy()
            for ti, it in enumerate(spec)])
        sizes = np.array([np.prod(it[1]) for it in spec], np.float64)
        rms = (norms / np.sqrt(sizes))[:, None]
        tiny = tiny | (np.abs(samp) < 1e-2 * rms) if s else (np.abs(samp) < 1e-2 * rms)
        d = np.abs(ps - f[f"s{s}_params_samp"])
        bound = 3e-7 if s == 0 else 1e-5  # after step 0: within one lr (no sign flips)
        assert np.all(d[~tiny] <= bound), f"step {s}: max {d[~tiny].max():.3e}"
        assert np.all(d[tiny] <= 2 * 1e-5 * (s + 1) * 1.01)
        assert tiny.mean() < 0.05
        rm = torch.cat([m.state_dict()[f"{n}.running_mean"].cpu() for n in O.BN_LAYERS]).numpy()
        rv = torch.cat([m.state_dict()[f"{n}.running_var"].cpu() for n in O.BN_LAYERS]).numpy()
        btol = 1e-4 if s == 0 else 1e-3
        np.testing.assert_allclose(rm, f[f"s{s}_running_mean"], rtol=btol, atol=btol)
        np.testing.assert_allclose(rv, f[f"s{s}_running_var"], rtol=btol, atol=btol)
        nbt = [int(m.state_dict()[f"{n}.num_batches_tracked"]) for n in O.BN_LAYERS]
        assert nbt == list(f[f"s{s}_nbt"])
    # eval mode (Trainer.validate / test): the oracle resynced from this path's parameters
    # and running statistics, at the north-star bar
    check_eval(m, O.forward, x.cpu(), t.cpu())


def _to64(d):
    return {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in d.items()}


def test_train_steps_strict_resync():
    """Per-step parity over 3 steps at lr 1e-4: before every step the oracle restarts from
    this path's current parameters, BN buffers and Adam moments (no trajectory drift).

    Gradients are judged against the fp64 evaluation of the same graph.  Any fp32
    evaluation flips a few ReLU masks whose pre-activation is within ~1e-6 of zero (e.g.
    step 0 here: one of decoder1's 262144 conv outputs is 2.7e-6 in fp64, <= 0 on this path),
    and one flip near the head moves every gradient upstream of it by ~1e-3 relative -- the
    fp32 reference shows the same ~1.5e-3 from its own flips in decoder2 (tools/diag_step0.py).
    So per step every HIP gradient must be within 2x the fp32 reference's worst per-tensor
    error, floored at FLIP_TOL at step 0 and at the SURVEY.md §8c bar GRAD_TOL once flips
    compound (steps 1-2, measured up to 5.2e-3); at step 0, where no flip reaches the head
    and final block,
    those tensors are held to 2x the fp32 error on that tensor + 1e-5."""
    import unet_hip
    P = O.make_params(42)
    x, t = inputs(1, 2, 64, 64)
    m = hip_model(P, DEV)
    opt = unet_hip.HipAdamW(m.parameters(), lr=1e-4)
    ref_opt = O.AdamWState(P, lr=1e-4)
    for s in range(3):
        Pc = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
        Bc = {k: v.detach().cpu().clone() for k, v in m.named_buffers()}
        r64 = O.train_step(_to64(Pc), _to64(Bc), None, x.double(), t.double())
        if s:
            for k, p in m.named_parameters():
                ref_opt.m[k] = opt.state[p]["exp_avg"].detach().cpu().clone()
                ref_opt.v[k] = opt.state[p]["exp_avg_sq"].detach().cpu().clone()
        ref_opt.step_count = s
        ref = O.train_step(Pc, Bc, ref_opt, x, t)
        logits, losses, loss = _step(m, opt, x.to(DEV), t.to(DEV))
        assert rel_max(logits.cpu().numpy(), ref["logits"].numpy()) <= LOGIT_TOL, f"step {s}"
        assert abs(loss.item() - ref["loss"].item()) <= 1e-5
        e_hip = grad_errors(m, r64["grads"])
        e32 = {k: norm_rel(g, r64["grads"][k]) for k, g in ref["grads"].items()}
        env = max(2 * max(e32.values()), FLIP_TOL if s == 0 else GRAD_TOL)
        for k in e32:
            assert e_hip[k] <= env, f"step {s} {k}: hip {e_hip[k]:.2e}, envelope {env:.2e}"
            if s == 0 and k.startswith("final."):
                assert e_hip[k] <= 2 * e32[k] + 1e-5, f"step {s} {k}: hip {e_hip[k]:.2e} vs {e32[k]:.2e}"


def test_full_grads_vs_oracle_64():
    """Every element of every gradient vs the oracle (not just the fixture samples)."""
    P = O.make_params(42)
    x, t = inputs(1, 2, 64, 64)
    ref = O.train_step(P, O.init_buffers(), None, x, t)
    m = hip_model(P, DEV)
    import unet_hip
    logits = m(x.to(DEV))
    losses = unet_hip.seg_losses(logits, t.to(DEV))
    (losses[0] + losses[1]).backward()
    errs = grad_errors(m, ref["grads"])
    worst = max(errs, key=errs.get)
    assert errs[worst] <= GRAD_TOL, f"{worst}: {errs[worst]:.3e}"


def test_b2_256_matches_golden(golden_dir):
    import unet_hip
    f = _golden(golden_dir, "unet_b2_256.npz")
    m = hip_model(O.make_params(42), DEV)
    x, t = inputs(2, 2, 256, 256)
    logits = m(x.to(DEV))
    losses = unet_hip.seg_losses(logits, t.to(DEV))
    loss = losses[0] + losses[1]
    loss.backward()
    flat = logits.detach().reshape(-1).cpu().numpy()
    mx = float(f["logit_max_abs"])
    assert np.max(np.abs(flat[f["logit_idx"]] - f["logit_samp"])) <= LOGIT_TOL * mx
    assert abs(np.abs(flat).max() - mx) <= LOGIT_TOL * mx
    bits = np.unpackbits(f["mask_bits"])[:flat.size]
    mask = (1 / (1 + np.exp(-flat.astype(np.float64))) > 0.5).astype(np.uint8)
    diff = mask != bits
    assert diff.sum() == 0 or np.all(np.abs(flat[diff]) <= 1e-3 * mx), f"{diff.sum()} mask bits"
    assert abs(loss.item() - float(f["loss"])) <= 1e-5
    for ti, (name, p) in enumerate(m.named_parameters()):
        n = p.grad.detach().double().norm().item()
        assert abs(n - f["grad_norm"][ti]) <= GRAD_TOL * f["grad_norm"][ti], name


def test_negative_gamma_matches_golden(golden_dir):
    """BN gamma < 0 before max-pool (max of BN(y), not BN of max(y)) and 2x2 bottleneck."""
    import unet_hip
    f = _golden(golden_dir, "unet_neg_32.npz")
    m = hip_model(O.make_params(5, -1.0, 1.0), DEV)
    x, t = inputs(4, 2, 32, 32)
    logits = m(x.to(DEV))
    losses = unet_hip.seg_losses(logits, t.to(DEV))
    (losses[0] + losses[1]).backward()
    assert rel_max(logits.detach().cpu().numpy(), f["logits"]) <= LOGIT_TOL
    for ti, (name, p) in enumerate(m.named_parameters()):
        n = p.grad.detach().double().norm().item()
        assert abs(n - f["grad_norm"][ti]) <= GRAD_TOL * f["grad_norm"][ti], name


@pytest.mark.parametrize("shape", [(4, 1, 96, 80), (3, 1, 97, 101), (2, 1, 512, 512)])
def test_losses_and_grads_vs_torch(shape):
    """Fused BCE/Dice/FocalTversky kernel vs torch fp32 ops (incl. soft targets, mixup).  Shapes:
    one chunk per sample; (r06) two chunks of an odd size (the scalar loop); 64 chunks per
    sample (config 4's 512^2 logits)."""
    import unet_hip
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(*shape, generator=g) * 4).to(DEV)
    t = torch.rand(*shape, generator=g).to(DEV)  # soft targets
    w = torch.tensor([0.7, 1.3, 0.5], device=DEV)
    xr = x.clone().requires_grad_(True)
    pr = torch.sigmoid(xr)
    bce = torch.nn.functional.binary_cross_entropy_with_logits(xr, t)
    pf, tf = pr.view(shape[0], -1), t.view(shape[0], -1)
    dice = 1 - ((2 * (pf * tf).sum(1) + 1) / (pf.sum(1) + tf.sum(1) + 1)).mean()
    TP = (pr * t).sum()
    FP = (pr * (1 - t)).sum()
    FN = ((1 - pr) * t).sum()
    ti = (TP + 1e-6) / (TP + 0.4 * FP + 0.6 * FN + 1e-6)
    focal = (1 - ti) ** 2.0
    (w[0] * bce + w[1] * dice + w[2] * focal).backward()
    xh = x.clone().requires_grad_(True)
    l = unet_hip.seg_losses(xh, t)
    (w * l).sum().backward()
    ref = torch.stack([bce, dice, focal]).detach()
    assert torch.allclose(l.detach(), ref, rtol=1e-5, atol=1e-6), (l, ref)
    assert norm_rel(xh.grad.cpu(), xr.grad.cpu()) <= 1e-4


def test_adamw_vs_torch():
    import unet_hip
    g = torch.Generator().manual_seed(5)
    p0 = torch.randn(1000003, generator=g).to(DEV)
    pa = torch.nn.Parameter(p0.clone())
    pb = torch.nn.Parameter(p0.clone())
    oa = torch.optim.AdamW([pa], lr=1e-3, foreach=False)
    ob = unet_hip.HipAdamW([pb], lr=1e-3)
    for _ in range(4):
        gr = torch.randn(1000003, generator=g).to(DEV)
        pa.grad = gr.clone()
        pb.grad = gr.clone()
        oa.step()
        ob.step()
    assert torch.max(torch.abs(pa - pb)).item() <= 1e-6


class _IeeeSqrtAdamW(O.AdamWState):
    """The oracle's AdamW (torch's CPU ops, op for op) with a correctly rounded sqrt: this
    host's vectorised torch.sqrt is 1 ulp low on ~0.7 % of fp32 inputs (measured against
    IEEE sqrt; a host-library property, not part of the algorithm)."""

    def step(self, params, grads):
        import math
        self.step_count += 1
        b1, b2 = self.betas
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        step_size = self.lr / bc1
        bc2_sqrt = math.sqrt(bc2)
        with torch.no_grad():
            for k, p in params.items():
                g = grads[k]
                p.mul_(1 - self.lr * self.wd)
                self.m[k].lerp_(g, 1 - b1)
                self.v[k].mul_(b2).addcmul_(g, g, value=1 - b2)
                sq = torch.from_numpy(np.sqrt(self.v[k].numpy()))
                denom = (sq / bc2_sqrt).add_(self.eps)
                p.addcdiv_(self.m[k], denom, value=-step_size)


@pytest.mark.parametrize("lr,wd,betas", [(1e-5, 1e-2, (0.9, 0.999)), (1e-3, 1e-2, (0.9, 0.999)),
                                         (3e-4, 0.1, (0.8, 0.99)), (1e-3, 0.0, (0.3, 0.9))])
def test_adamw_bitwise_vs_oracle(lr, wd, betas):
    """The native AdamW vs the oracle's (torch's _single_tensor_adam CPU ops, utils/
    trainer.py:41,92) from IDENTICAL p, g, m, v at every one of 4 steps, over a flat arena
    of 2^20 + 3 floats (16-B-vectorised kernel on the aligned body).

    * exp_avg and exp_avg_sq: bit-identical on every element;
    * params: bit-identical to the oracle's op sequence with a correctly rounded sqrt
      (_IeeeSqrtAdamW) on every element, and within 1 ulp (of the larger addend) of the
      pure-torch oracle, whose only differences are the elements where the host's sqrt is
      not correctly rounded."""
    import unet_hip
    n = (1 << 20) + 3
    gen = torch.Generator().manual_seed(int(lr * 1e6) + int(wd * 100))
    p = (torch.randn(n, generator=gen) * 0.05).float()
    ref = O.AdamWState({"a": p.clone()}, lr=lr, betas=betas, weight_decay=wd)
    ieee = _IeeeSqrtAdamW({"a": p.clone()}, lr=lr, betas=betas, weight_decay=wd)
    pd = torch.nn.Parameter(p.clone().to(DEV))
    opt = unet_hip.HipAdamW([pd], lr=lr, betas=betas, weight_decay=wd)
    for s in range(4):
        scale = 10.0 ** torch.empty(n).uniform_(-7, -1, generator=gen)
        g = torch.randn(n, generator=gen) * scale
        # identical state going in: the device copy of the oracle's p, m, v
        P_ref, P_ieee = {"a": p.clone()}, {"a": p.clone()}
        ref.m["a"], ref.v["a"] = ieee.m["a"].clone(), ieee.v["a"].clone()
        ref.step_count = ieee.step_count
        m_in, v_in = ieee.m["a"].clone(), ieee.v["a"].clone()
        with torch.no_grad():
            pd.copy_(p.to(DEV))
        if s:
            opt.state[pd]["exp_avg"].copy_(m_in.to(DEV))
            opt.state[pd]["exp_avg_sq"].copy_(v_in.to(DEV))
        pd.grad = g.to(DEV)
        ref.step(P_ref, {"a": g})
        ieee.step(P_ieee, {"a": g})
        opt.step()
        torch.cuda.synchronize()
        got_p = pd.detach().cpu()
        got_m = opt.state[pd]["exp_avg"].cpu()
        got_v = opt.state[pd]["exp_avg_sq"].cpu()
        assert torch.equal(got_m, ref.m["a"]), f"step {s}: exp_avg differs"
        assert torch.equal(got_v, ref.v["a"]), f"step {s}: exp_avg_sq differs"
        assert torch.equal(got_p, P_ieee["a"]), \
            f"step {s}: {(got_p != P_ieee['a']).sum().item()} params differ from the IEEE-sqrt oracle"
        diff = got_p != P_ref["a"]
        v = ref.v["a"]
        hs, ies = torch.sqrt(v), torch.from_numpy(np.sqrt(v.numpy()))
        host_sqrt_off = hs != ies
        assert bool(torch.all(host_sqrt_off[diff])), "a difference not explained by the host sqrt"
        # a k-ulp error of the host's sqrt is a relative error of k * 2^-23 in the denominator,
        # so at most a few k * 2^-23 of the update u = p_new - p * decay (plus the final
        # rounding of p_new): bound it at 8 k * 2^-23 |u| + 1 ulp of p_new
        k = int((hs.view(torch.int32).long() - ies.view(torch.int32).long()).abs().max())
        u = P_ieee["a"].double() - p.double() * (1 - lr * wd)
        dp = (got_p.double() - P_ref["a"].double()).abs()
        bound = 8 * k * 2.0 ** -23 * u.abs() + torch.from_numpy(np.spacing(P_ref["a"].abs().numpy())).double()
        assert bool(torch.all(dp <= bound)), \
            f"step {s}: {float((dp / bound).max()):.2f} x the bound, host sqrt up to {k} ulp"
        print(f"step {s}: {int(diff.sum())} of {n} params differ from the torch-CPU oracle "
              f"(host sqrt inexact on {int(host_sqrt_off.sum())}, by up to {k} ulp)")
        p = P_ieee["a"]


def _focal_step(m, opt, x, t):
    import unet_hip
    opt.zero_grad()
    logits = m(x)
    losses = unet_hip.seg_losses(logits, t)
    loss = 1.0 * losses[0] + 0.0 * losses[1] + 1.0 * losses[2]  # main.py:43-46 defaults
    loss.backward()
    opt.step()
    return logits.detach(), losses.detach(), loss.detach()


def test_focal_default_mix_matches_golden(golden_dir):
    """The reference CLI's default loss (BCE 1 / Dice 0 / FocalTversky 1, main.py:43-46)
    over three training steps vs tests/golden/unet_focal_64.npz (the real
    FocalTverskyLoss of models/loss.py:26-46).  Step 0 at the strict bars; steps 1-2 at
    the trajectory-drift bars of test_train_steps_match_golden."""
    import unet_hip
    f = _golden(golden_dir, "unet_focal_64.npz")
    m = hip_model(O.make_params(42), DEV)
    opt = unet_hip.HipAdamW(m.parameters(), lr=1e-5)
    x, t = torch.from_numpy(f["x"]).to(DEV), torch.from_numpy(f["t"]).to(DEV)
    for s in range(3):
        p = f"s{s}_"
        logits, losses, loss = _focal_step(m, opt, x, t)
        tol = LOGIT_TOL if s == 0 else 2e-3
        assert rel_max(logits.cpu().numpy(), f[p + "logits"]) <= tol, f"step {s} logits"
        ltol = 1e-5 if s == 0 else 1e-4
        for i, k in enumerate(("bce", "dice", "focal")):
            assert abs(losses[i].item() - float(f[p + k])) <= ltol, (s, k)
        assert abs(loss.item() - float(f[p + "loss"])) <= ltol
        gtol = GRAD_TOL if s == 0 else 10 * GRAD_TOL
        norms = f[p + "grad_norm"]
        for ti, (name, prm) in enumerate(m.named_parameters()):
            n = prm.grad.detach().double().norm().item()
            assert abs(n - norms[ti]) <= gtol * norms[ti], (s, name)


def test_focal_full_grads_vs_oracle():
    """Every gradient element with FocalTversky in the loss (weights 1/1/1) vs the oracle."""
    P = O.make_params(42)
    x, t = inputs(21, 2, 64, 64)
    ref = O.train_step(P, O.init_buffers(), None, x, t, w_bce=1.0, w_dice=1.0, w_focal=1.0)
    m = hip_model(P, DEV)
    import unet_hip
    logits = m(x.to(DEV))
    losses = unet_hip.seg_losses(logits, t.to(DEV))
    (losses[0] + losses[1] + losses[2]).backward()
    assert abs(losses[2].item() - ref["focal"].item()) <= 1e-5
    errs = grad_errors(m, ref["grads"])
    worst = max(errs, key=errs.get)
    assert errs[worst] <= GRAD_TOL, f"{worst}: {errs[worst]:.3e}"


def test_eval_mode_parity_after_training():
    """Trainer.test / validate path (utils/trainer.py:130,206-250): eval-mode BN from the
    running statistics of three training steps, at 1e-4, masks and counts."""
    import unet_hip
    x, t = inputs(7, 4, 128, 96)
    m = hip_model(O.make_params(42), DEV)
    opt = unet_hip.HipAdamW(m.parameters(), lr=1e-4)
    for _ in range(3):
        _step(m, opt, x.to(DEV), t.to(DEV))
    nd = check_eval(m, O.forward, x, t)
    print(f"eval masks: {nd} near-boundary bits differ")


def test_mask_counts():
    import unet_hip
    g = torch.Generator().manual_seed(9)
    x = torch.randn(3, 1, 64, 48, generator=g).to(DEV)
    t = (torch.rand(3, 1, 64, 48, generator=g) > 0.6).float().to(DEV)
    rt = unet_hip.UNetRuntime.get(DEV)
    counts = torch.zeros(6, dtype=torch.int64, device=DEV)
    mask = torch.empty(x.shape, dtype=torch.uint8, device=DEV)
    rt.mask_counts(x, t, counts, mask)
    pm = (torch.sigmoid(x) > 0.5)
    tm = t.to(torch.uint8) == 1
    tb = t != 0
    want = [int((pm & tm).sum()), int((pm & ~tm).sum()), int((~pm & tm).sum()), int((~pm & ~tm).sum()),
            int((pm & tb).sum()), int((pm | tb).sum())]
    assert counts.cpu().tolist() == want
    assert torch.equal(mask.bool(), pm)


def test_full_size_vs_cpu_oracle():
    """bs=32, 1x256x256 (BASELINE config 2): forward and gradients vs the CPU oracle's step on
    the box's host threads (~15 s; the same functional graph on the GPU through torch/MIOpen
    spent ~110 s compiling its kernels on every fresh box)."""
    import unet_hip
    P = O.make_params(42)
    x, t = inputs(11, 32, 256, 256)
    ref = O.train_step(P, O.init_buffers(), None, x, t)
    m = hip_model(P, DEV)
    logits = m(x.to(DEV))
    losses = unet_hip.seg_losses(logits, t.to(DEV))
    (losses[0] + losses[1]).backward()
    assert rel_max(logits.detach().cpu().numpy(), ref["logits"].cpu().numpy()) <= LOGIT_TOL
    errs = grad_errors(m, {k: v.cpu() for k, v in ref["grads"].items()})
    worst = max(errs, key=errs.get)
    assert errs[worst] <= GRAD_TOL, f"{worst}: {errs[worst]:.3e}"


def test_determinism_full_size():
    """Two identical training forwards+backwards are bit-identical (no float atomics)."""
    import unet_hip
    P = O.make_params(42)
    x, t = inputs(12, 8, 256, 256)
    outs = []
    for _ in range(2):
        m = hip_model(P, DEV)
        logits = m(x.to(DEV))
        l = unet_hip.seg_losses(logits, t.to(DEV))
        (l[0] + l[1]).backward()
        outs.append((logits.detach().clone(), m.flat_params.grad if False else
                     m._state.grad_arena.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("out_ch,B,H,W", [(2, 2, 64, 128), (1, 1, 48, 80), (4, 3, 32, 32)])
def test_shapes_and_classes_vs_oracle(out_ch, B, H, W):
    """Non-square images, batch 1, H/W multiples of 16 that are not powers of two, and the
    multi-class head (models/model.py:6 out_channels; the losses flatten all classes like
    models/loss.py:19-20).  Small images at batch 1 leave the deep BatchNorms a handful of
    values per channel (15 at level 4 for 48x80), where a near-zero ReLU input flips under
    any fp32 rounding change: gradients are judged against fp64 within 2x the fp32
    oracle's own error over x and x * (1 + 1e-7) (as tests/test_gpu_res.py), floor 1e-2."""
    import unet_hip
    P = O.make_params(3, out_channels=out_ch)
    x, _ = inputs(6, B, H, W)
    t = (torch.rand(B, out_ch, H, W, generator=torch.Generator().manual_seed(1)) > 0.7).float()
    ref = O.train_step(P, O.init_buffers(), None, x, t)
    refp = O.train_step(P, O.init_buffers(), None, x * (1 + 1e-7), t)
    r64 = O.train_step(_to64(P), _to64(O.init_buffers()), None, x.double(), t.double())
    m = unet_hip.UNet(1, out_ch)
    sd = m.state_dict()
    for k, v in P.items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    logits = m(x.to(DEV))
    assert logits.shape == (B, out_ch, H, W)
    losses = unet_hip.seg_losses(logits, t.to(DEV))
    (losses[0] + losses[1]).backward()
    assert rel_max(logits.detach().cpu().numpy(), ref["logits"].numpy()) <= LOGIT_TOL
    assert abs((losses[0] + losses[1]).item() - ref["loss"].item()) <= 1e-5
    e32 = {k: max(norm_rel(g, r64["grads"][k]), norm_rel(refp["grads"][k], r64["grads"][k]))
           for k, g in ref["grads"].items()}
    env = max(2 * max(e32.values()), GRAD_TOL)
    errs = grad_errors(m, r64["grads"])
    worst = max(errs, key=errs.get)
    assert errs[worst] <= env, f"{worst}: {errs[worst]:.3e} (fp32 oracle {e32[worst]:.3e})"


@pytest.mark.parametrize("variant", ["model", "mod"])
def test_wgrad_row3_matches_one_tap_tiles(variant):
    """Option wgrad_row3=1 (the default) computes every eligible 3x3 weight gradient with the
    one-row-of-taps kernel (kernels_gemm.hip wgrad_row3_kernel: three taps per block from
    a halo-staged input row, a different split-K partition).  Same products, different
    summation grouping: every weight / bias gradient within 1e-5 norm-relative of the
    one-tap schedule, logits bit-identical (the forward does not change)."""
    import unet_hip
    from _helpers import hip_mod_model, options
    x, t = inputs(17, 8, 256, 256)
    outs = []
    for flag in (0, 1):
        if variant == "model":
            m = hip_model(O.make_params(42), DEV)
        else:
            from oracle import mod_ref_cpu as MO
            m = hip_mod_model(MO.make_params(5, base=64, depth=4), DEV, 64, 4)
        # (x3 = 0: the f32 MFMA weight gradients are the subject)
        with options(m.flatten_().rt, x3=0, wgrad_row3=flag):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        outs.append((logits.detach().clone(),
                     {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    assert torch.equal(outs[0][0], outs[1][0])
    worst = 0.0
    for k, g0 in outs[0][1].items():
        d = float((outs[1][1][k] - g0).norm() / max(float(g0.norm()), 1e-30))
        worst = max(worst, d)
        assert d <= 1e-5, (k, d)
    print(f"row3 vs one-tap worst grad norm-rel {worst:.2e}")


@pytest.mark.parametrize("variant,B,H,W", [("model", 2, 64, 64), ("model", 8, 256, 256),
                                           ("model", 1, 48, 80), ("mod", 2, 128, 64),
                                           ("res", 2, 64, 64)])
def test_pipe_gemm_bit_identical(variant, B, H, W):
    """Row-GEMM tiles 18, 19, 25, 26 (kernels_gemm_pipe.hip: the software-pipelined schedule
    of the 128x128 / 128x64 f32 tiles, global loads two chunks ahead, 18 the default;
    25 / 26: 128x64 at three blocks per CU, the N = 64 dgrad / ConvT-dgrad defaults) walk K in
    the same order with the same prologue arithmetic and the same epilogues as the
    register-staged rowgemm_kernel tiles (4, 0, 1), so a training step -- logits and the
    whole gradient arena -- is bit-identical across the schedules.  48x80 has M
    tiles that end past M (rows masked in the gather and the guarded epilogue path); the
    ResUNet covers the 1x1 skip GEMMs (E_RESID) and E_ADD, the ConvTranspose GEMMs run in
    every variant."""
    import unet_hip
    from _helpers import hip_mod_model, options
    from oracle import mod_ref_cpu as MO
    x, t = inputs(43, B, H, W)
    outs = []
    for tiles in ((4, 0, 1, 0), (18, 18, 19, 18), (18, 4, 25, 26), (4, 18, 26, 25)):
        if variant == "model":
            m = hip_model(O.make_params(42), DEV)
        elif variant == "mod":
            m = hip_mod_model(MO.make_params(5, 64, 3), DEV, 64, 3)
        else:
            m = unet_hip.ResUNet(1, 1, base_filters=64, depth=3)
            sd = m.state_dict()
            sd.update({k: v.clone() for k, v in MO.res_make_params(42, 64, 3).items()})
            m.load_state_dict(sd)
            m = m.to(DEV).train()
        with options(m.flatten_().rt, x3=0, tile_n128=tiles[0], tile_n128_dgrad=tiles[1],
                     tile_n64=tiles[2], tile_n64_dgrad=tiles[2], tile_convt64=tiles[2],
                     tile_convt_dgrad=tiles[3]):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        outs.append((logits.detach().clone(), m._state.grad_arena.clone()))
        del m
    for i in range(1, len(outs)):
        assert torch.equal(outs[0][0], outs[i][0]), i
        d = (outs[0][1] - outs[i][1]).abs().max().item()
        assert torch.equal(outs[0][1], outs[i][1]), (i, d)


@pytest.mark.parametrize("B,H,W", [(2, 64, 64), (8, 256, 256), (1, 48, 80)])
def test_dz_in_wgrad_bit_identical(B, H, W):
    """Option dz_in_wgrad: the weight gradient's B' loader forms the BN-backward dz from do
    and y (the same bn_dz4 helper as the bn_dz pass) and its first A'-tile blocks store it
    for the dgrad, so the bn_dz pass disappears.  The stored dz, the bias column sums and
    every gradient are the same bits as with the separate pass (models/model.py order)."""
    import unet_hip
    from _helpers import options
    x, t = inputs(47, B, H, W)
    outs = []
    for flag in (0, 1 << 20):  # off / every layer (default: Cin <= 256)
        m = hip_model(O.make_params(42), DEV)
        with options(m.flatten_().rt, x3=0, dz_in_wgrad=flag):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        outs.append((logits.detach().clone(), m._state.grad_arena.clone()))
        del m
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1]), (outs[0][1] - outs[1][1]).abs().max().item()


def test_adamw_resume_from_state_dict_matches_uninterrupted():
    """HipAdamW honours optimizer.load_state_dict on its flat path: two steps, save the
    state dict, a fresh optimizer over fresh parameters loads it (and the parameters), then
    two more steps -- bit-identical params, exp_avg, exp_avg_sq to the uninterrupted run,
    which itself keeps m / v bit-identical to the oracle (torch's _single_tensor_adam)."""
    import unet_hip
    sizes = [(64, 3, 3, 3), (64,), (1000, 7)]
    n = sum(int(np.prod(s)) for s in sizes)
    gen = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=gen) * 0.05
    grads = [torch.randn(n, generator=gen) * 10.0 ** torch.empty(n).uniform_(-6, -1, generator=gen)
             for _ in range(4)]

    def make(flat_init):
        flat = flat_init.clone().to(DEV)
        gflat = torch.zeros_like(flat)
        ps, off = [], 0
        for s in sizes:
            k = int(np.prod(s))
            ps.append(torch.nn.Parameter(flat[off:off + k].view(s)))
            off += k
        return flat, gflat, ps

    def run(opt, flat, gflat, ps, gs):
        for g in gs:
            gflat.copy_(g.to(DEV))
            off = 0
            for p in ps:
                p.grad = gflat[off:off + p.numel()].view(p.shape)
                off += p.numel()
            opt.step()

    fa, ga, pa = make(p0)
    oa = unet_hip.HipAdamW(pa, lr=1e-3)
    ref = O.AdamWState({"a": p0.clone()}, lr=1e-3)
    run(oa, fa, ga, pa, grads[:2])
    sd = {k: v for k, v in oa.state_dict().items()}
    sd = torch.utils._pytree.tree_map(lambda v: v.detach().cpu().clone() if torch.is_tensor(v) else v, sd)
    mid = fa.detach().cpu().clone()
    run(oa, fa, ga, pa, grads[2:])
    fb, gb, pb = make(mid)
    ob = unet_hip.HipAdamW(pb, lr=1e-3)
    ob.load_state_dict(sd)
    run(ob, fb, gb, pb, grads[2:])
    torch.cuda.synchronize()
    assert torch.equal(fa.cpu(), fb.cpu()), "resumed params differ from the uninterrupted run"
    for p, q in zip(pa, pb):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(oa.state[p][k].cpu(), ob.state[q][k].cpu()), k
        assert float(ob.state[q]["step"]) == 4.0
    # the moments of the uninterrupted run vs the oracle's op sequence
    P = {"a": p0.clone()}
    for g in grads:
        ref.step(P, {"a": g})
    m = torch.cat([oa.state[p]["exp_avg"].reshape(-1).cpu() for p in pa])
    v = torch.cat([oa.state[p]["exp_avg_sq"].reshape(-1).cpu() for p in pa])
    assert torch.equal(m, ref.m["a"]) and torch.equal(v, ref.v["a"])


def test_bucket_event_exported_for_non_torch_callers():
    """unet_bucket_event (include/unet_hip.h): the raw hipEvent_t per gradient bucket that a
    caller driving RCCL on its own streams waits on.  Each bucket's slice, copied on a
    fresh stream that only waited (hipStreamWaitEvent through the HIP runtime itself, no
    torch stream sync) on that bucket's event, equals the final gradient arena."""
    import ctypes
    import unet_hip
    hip = ctypes.CDLL("libamdhip64.so")  # the process's one HIP runtime (torch's)
    hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    x, t = inputs(61, 4, 128, 128)
    m = hip_model(O.make_params(42), DEV)
    rt = m.flatten_().rt
    logits = m(x.to(DEV))
    l = unet_hip.seg_losses(logits, t.to(DEV))
    (l[0] + l[1]).backward()  # enqueued; no host sync before the waits below
    arena = m._state.grad_arena
    copies = []
    for b, (off, n) in enumerate(rt.buckets):
        s = torch.cuda.Stream(device=DEV)
        ev = rt.bucket_event(b)
        assert ev, "null event"
        assert hip.hipStreamWaitEvent(ctypes.c_void_p(s.cuda_stream), ctypes.c_void_p(ev), 0) == 0
        with torch.cuda.stream(s):
            copies.append(arena[off:off + n].clone())
    torch.cuda.synchronize()
    for (off, n), c in zip(rt.buckets, copies):
        assert torch.equal(c, arena[off:off + n])


def _train_steps(m, opt, batches):
    import unet_hip
    out = []
    for x, t in batches:
        opt.zero_grad()
        logits = m(x.to(DEV))
        losses = unet_hip.seg_losses(logits, t.to(DEV))
        (losses[0] + losses[1]).backward()
        opt.step()
        torch.cuda.synchronize()
        out.append(logits.detach().clone())
    return out


@pytest.mark.parametrize("variant", ["model", "mod_bf16"])
def test_adamw_repack_bit_identical(variant, monkeypatch):
    """unet_adamw_repack (r06): HipAdamW over a HIP model's whole arena updates each 3x3 / ConvT
    weight tile and packs it into the context's GEMM images in one pass, and the next forward
    reads those images instead of repacking.  Three training steps must be bit-identical --
    logits of every step, the parameter arena, exp_avg and exp_avg_sq -- to the unfused path
    (unet_adamw, then the forward's own repack): models/model.py UNet (f32 on the x3 images) and
    config 4's mod.py UNet(128, 5) on bf16 images."""
    import unet_hip
    import unet_hip.module as UM
    from oracle import mod_ref_cpu as MO
    H = 64 if variant == "model" else 128
    batches = [inputs(90 + k, 2, H, H) for k in range(3)]
    res = {}
    for fused in (1, 0):
        if not fused:
            monkeypatch.setattr(UM, "arena_owner", lambda flat: None)
        if variant == "model":
            m = hip_model(O.make_params(42), DEV)
        else:
            m = unet_hip.ModUNet(1, 1, base_filters=128, depth=5, mfma_dtype="bf16")
            sd = m.state_dict()
            sd.update({k: v.clone() for k, v in MO.make_params(61, 128, 5).items()})
            m.load_state_dict(sd)
            m = m.to(DEV).train()
        opt = unet_hip.HipAdamW(m.parameters(), lr=1e-3)
        lg = _train_steps(m, opt, batches)
        st = m.flatten_()
        p0 = next(m.parameters())
        res[fused] = (lg, st.param_arena.clone(), opt.state[p0]["exp_avg"].clone(),
                      opt.state[p0]["exp_avg_sq"].clone())
        del m, opt
    for k, (a, b) in enumerate(zip(res[1][0], res[0][0])):
        assert torch.equal(a, b), f"step {k} logits"
    assert torch.equal(res[1][1], res[0][1]), (res[1][1] - res[0][1]).abs().max().item()
    assert torch.equal(res[1][2], res[0][2]) and torch.equal(res[1][3], res[0][3])


def test_adamw_repack_invalidation():
    """The fused path's weight images follow the parameters: a torch in-place write after a
    fused step (load_state_dict-style; the parameter's version counter moves) is seen by the
    next forward (it repacks), so is a write through `.data` declared with params_changed(), and
    a backward whose forward read the images refuses to run after another fused step rewrote
    them."""
    import unet_hip
    from unet_hip._lib import HipError
    x, t = inputs(95, 2, 64, 64)
    m = hip_model(O.make_params(42), DEV)
    opt = unet_hip.HipAdamW(m.parameters(), lr=1e-3)
    _train_steps(m, opt, [(x, t)])
    # forward on the fused images, then a fused step in between, then its backward
    logits = m(x.to(DEV))
    losses = unet_hip.seg_losses(logits, t.to(DEV))
    opt.step()  # the grads of the first step are still there: a fused repack
    with pytest.raises(HipError):
        (losses[0] + losses[1]).backward()
    with torch.no_grad():
        m.encoder2[0].weight.mul_(0.5)  # bumps the arena's version counter
    got = m(x.to(DEV)).detach().clone()
    ref = hip_model({k: v.detach().cpu() for k, v in m.named_parameters()}, DEV)
    want = ref(x.to(DEV)).detach()
    assert torch.equal(got, want)
    del ref
    # writes through .data bypass the version counters: declared with params_changed()
    _train_steps(m, opt, [(x, t)])
    m.encoder3[0].weight.data.mul_(-1.0)
    m.params_changed()
    got = m(x.to(DEV)).detach().clone()
    ref = hip_model({k: v.detach().cpu() for k, v in m.named_parameters()}, DEV)
    want = ref(x.to(DEV)).detach()
    assert torch.equal(got, want)
