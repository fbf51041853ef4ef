"""Pin the CPU oracle (oracle/unet_ref_cpu.py) against the reference's own outputs.

The fixtures in tests/golden/ were written by tools/gen_golden.py, which imports the
unmodified reference (models/model.py, models/loss.py, torch AdamW as
utils/trainer.py:41 builds it) in the build container.  On the same machine the
restatement is bit-identical; elsewhere (different CPU, different oneDNN kernels) it
agrees to fp32 rounding, which is what these tolerances allow.
"""
import os

import numpy as np
import pytest
import torch

from oracle import unet_ref_cpu as O
from oracle import weights as W


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def _grad_stats(grads, spec):
    norms, sums, samp = [], [], []
    for t, item in enumerate(spec):
        g = grads[item[0]].double().reshape(-1)
        idx = np.floor(W.uniform(7, 3000 + t, 64) * g.numel()).astype(np.int64)
        norms.append(g.norm().item())
        sums.append(g.sum().item())
        samp.append(g[torch.from_numpy(idx)].numpy())
    return np.array(norms), np.array(sums), np.stack(samp)


def _check_grads(g, norms, sums, samp, rtol):
    n, s, sm = g
    np.testing.assert_allclose(n, norms, rtol=rtol, atol=0)
    scale = norms[:, None]
    assert np.all(np.abs(sm - samp) <= rtol * scale + 1e-30)
    assert np.all(np.abs(s - sums) <= rtol * norms * 100)


def test_param_spec_and_count():
    spec = O.param_spec()
    assert len(spec) == 82
    assert sum(int(np.prod(s[1])) for s in spec) == 31_042_369
    assert O.train_flops_per_image(256, 256) == 288_475_840_512


def test_oracle_b2_64_three_steps(golden_dir):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    f = _load(golden_dir, "unet_b2_64.npz")
    P = O.make_params(42)
    B = O.init_buffers()
    opt = O.AdamWState(P, lr=1e-5)
    x, t = torch.from_numpy(f["x"]), torch.from_numpy(f["t"])
    np.testing.assert_array_equal(f["x"], W.make_input(1, 2, 1, 64, 64))
    np.testing.assert_array_equal(f["t"], W.make_target(1, 2, 64, 64))
    spec = O.param_spec()
    for s in range(3):
        r = O.train_step(P, B, opt, x, t)
        ref = f[f"s{s}_logits"]
        assert np.max(np.abs(r["logits"].numpy() - ref)) <= 1e-5 * np.max(np.abs(ref))
        np.testing.assert_array_equal(O.mask_readout(r["logits"]).numpy(), f[f"s{s}_mask"])
        assert abs(r["bce"].item() - float(f[f"s{s}_bce"])) < 1e-6
        assert abs(r["dice"].item() - float(f[f"s{s}_dice"])) < 1e-6
        _check_grads(_grad_stats(r["grads"], spec), f[f"s{s}_grad_norm"], f[f"s{s}_grad_sum"],
                     f[f"s{s}_grad_samp"], rtol=1e-4)
        psamp = np.stack([P[it[0]].reshape(-1)[torch.from_numpy(
            np.floor(W.uniform(7, 3000 + ti, 64) * P[it[0]].numel()).astype(np.int64))].numpy()
            for ti, it in enumerate(spec)])
        np.testing.assert_allclose(psamp, f[f"s{s}_params_samp"], rtol=0, atol=1e-7)
        rm = np.concatenate([B[f"{n}.running_mean"].numpy() for n in O.BN_LAYERS])
        rv = np.concatenate([B[f"{n}.running_var"].numpy() for n in O.BN_LAYERS])
        np.testing.assert_allclose(rm, f[f"s{s}_running_mean"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(rv, f[f"s{s}_running_var"], rtol=1e-5, atol=1e-6)
        assert [B[f"{n}.num_batches_tracked"].item() for n in O.BN_LAYERS] == list(f[f"s{s}_nbt"])
    with torch.no_grad():
        ev = O.forward(x, P, B, training=False).numpy()
    assert np.max(np.abs(ev - f["eval_logits"])) <= 1e-5 * np.max(np.abs(f["eval_logits"]))


def test_oracle_b2_256(golden_dir):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    f = _load(golden_dir, "unet_b2_256.npz")
    P = O.make_params(42)
    B = O.init_buffers()
    x = torch.from_numpy(W.make_input(2, 2, 1, 256, 256))
    t = torch.from_numpy(W.make_target(2, 2, 256, 256))
    r = O.train_step(P, B, None, x, t)
    flat = r["logits"].reshape(-1).numpy()
    assert np.max(np.abs(flat[f["logit_idx"]] - f["logit_samp"])) <= 1e-5 * float(f["logit_max_abs"])
    bits = np.packbits(O.mask_readout(r["logits"]).numpy().reshape(-1))
    np.testing.assert_array_equal(bits, f["mask_bits"])
    assert abs(r["loss"].item() - float(f["loss"])) < 1e-6
    _check_grads(_grad_stats(r["grads"], O.param_spec()), f["grad_norm"], f["grad_sum"],
                 f["grad_samp"], rtol=1e-4)


def test_oracle_dp2_64(golden_dir):
    f = _load(golden_dir, "unet_dp2_64.npz")
    P = O.make_params(42)
    B = O.init_buffers()
    x = torch.from_numpy(W.make_input(3, 4, 1, 64, 64))
    t = torch.from_numpy(W.make_target(3, 4, 64, 64))
    r = O.train_step(P, B, None, x, t, shards=2)
    assert abs(r["loss"].item() - float(f["loss"])) < 1e-6
    _check_grads(_grad_stats(r["grads"], O.param_spec()), f["grad_norm"], f["grad_sum"],
                 f["grad_samp"], rtol=1e-4)


def test_oracle_negative_gamma(golden_dir):
    f = _load(golden_dir, "unet_neg_32.npz")
    P = O.make_params(5, -1.0, 1.0)
    B = O.init_buffers()
    x = torch.from_numpy(W.make_input(4, 2, 1, 32, 32))
    t = torch.from_numpy(W.make_target(4, 2, 32, 32))
    r = O.train_step(P, B, None, x, t)
    ref = f["logits"]
    assert np.max(np.abs(r["logits"].numpy() - ref)) <= 1e-5 * np.max(np.abs(ref))
    _check_grads(_grad_stats(r["grads"], O.param_spec()), f["grad_norm"], f["grad_sum"],
                 f["grad_samp"], rtol=1e-4)


def test_mod_param_spec_and_flops():
    from oracle import mod_ref_cpu as MO
    spec = MO.param_spec(1, 1, 128, 5)
    assert sum(int(np.prod(s[1])) for s in spec) == 497_438_849
    assert MO.train_flops_per_image(512, 512, 128, 5) == 5_709_420_822_528  # §8d config 4


@pytest.mark.parametrize("tag,seed,lo,hi", [("", 42, 0.5, 1.5), ("neg_", 5, -1.0, 1.0)])
def test_oracle_mod_d3_two_steps(golden_dir, tag, seed, lo, hi):
    """models/mod.py UNet(base 64, depth 3): BN->ReLU, [skip, up], bias-free convs."""
    from oracle import mod_ref_cpu as MO
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    f = _load(golden_dir, "mod_d3_64.npz")
    P = MO.make_params(seed, 64, 3, lo, hi)
    B = MO.init_buffers(64, 3)
    opt = O.AdamWState(P, lr=1e-4)
    x = torch.from_numpy(W.make_input(11, 2, 1, 64, 64))
    t = torch.from_numpy(W.make_target(11, 2, 64, 64))
    spec = MO.param_spec(1, 1, 64, 3)
    names = [n for n, _ in MO.bn_layers(64, 3)]
    for s in range(2):
        p = f"{tag}s{s}_"
        r = MO.train_step(P, B, opt, x, t, depth=3)
        ref = f[p + "logits"]
        assert np.max(np.abs(r["logits"].numpy() - ref)) <= 1e-5 * np.max(np.abs(ref))
        assert abs(r["loss"].item() - float(f[p + "loss"])) < 1e-6
        _check_grads(_grad_stats(r["grads"], spec), f[p + "grad_norm"], f[p + "grad_sum"],
                     f[p + "grad_samp"], rtol=1e-4)
        rm = np.concatenate([B[f"{n}.running_mean"].numpy() for n in names])
        np.testing.assert_allclose(rm, f[p + "running_mean"], rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        ev = MO.make_forward(3)(x, P, B, training=False).numpy()
    assert np.max(np.abs(ev - f[tag + "eval_logits"])) <= 1e-5 * np.max(np.abs(f[tag + "eval_logits"]))


def test_oracle_mod_config4_arch(golden_dir):
    """The config-4 architecture (base 128, depth 5, 497 M params) at B=2 64x64."""
    from oracle import mod_ref_cpu as MO
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    f = _load(golden_dir, "mod_c4_64.npz")
    P = MO.make_params(42, 128, 5)
    x = torch.from_numpy(W.make_input(12, 2, 1, 64, 64))
    t = torch.from_numpy(W.make_target(12, 2, 64, 64))
    r = MO.train_step(P, MO.init_buffers(128, 5), None, x, t, depth=5)
    assert np.max(np.abs(r["logits"].numpy() - f["logits"])) <= 1e-5 * np.max(np.abs(f["logits"]))
    assert abs(r["loss"].item() - float(f["loss"])) < 1e-6
    _check_grads(_grad_stats(r["grads"], MO.param_spec(1, 1, 128, 5)), f["grad_norm"],
                 f["grad_sum"], f["grad_samp"], rtol=1e-4)


def test_oracle_res_d3_two_steps(golden_dir):
    """models/mod.py ResUNet(base 64, depth 3) -- residual blocks relu(conv(x) + skip(x))."""
    from oracle import mod_ref_cpu as MO
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    f = _load(golden_dir, "res_d3_64.npz")
    P = MO.res_make_params(42, 64, 3)
    B = MO.res_init_buffers(64, 3)
    opt = O.AdamWState(P, lr=1e-4)
    x = torch.from_numpy(W.make_input(13, 2, 1, 64, 64))
    t = torch.from_numpy(W.make_target(13, 2, 64, 64))
    spec = MO.res_param_spec(1, 1, 64, 3)
    names = [n for n, _ in MO.res_bn_layers(64, 3)]
    for s in range(2):
        p = f"s{s}_"
        r = MO.res_train_step(P, B, opt, x, t, depth=3)
        ref = f[p + "logits"]
        assert np.max(np.abs(r["logits"].numpy() - ref)) <= 1e-5 * np.max(np.abs(ref))
        assert abs(r["loss"].item() - float(f[p + "loss"])) < 1e-6
        _check_grads(_grad_stats(r["grads"], spec), f[p + "grad_norm"], f[p + "grad_sum"],
                     f[p + "grad_samp"], rtol=1e-4)
        rm = np.concatenate([B[f"{n}.running_mean"].numpy() for n in names])
        np.testing.assert_allclose(rm, f[p + "running_mean"], rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        ev = MO.make_res_forward(3)(x, P, B, training=False).numpy()
    assert np.max(np.abs(ev - f["eval_logits"])) <= 1e-5 * np.max(np.abs(f["eval_logits"]))


def test_oracle_focal_default_mix_three_steps(golden_dir):
    """The reference CLI's default loss mix (main.py:43-46: BCE 1, Dice 0, FocalTversky 1)
    over three AdamW steps (tests/golden/unet_focal_64.npz, real FocalTverskyLoss)."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    f = _load(golden_dir, "unet_focal_64.npz")
    P = O.make_params(42)
    B = O.init_buffers()
    opt = O.AdamWState(P, lr=1e-5)
    x, t = torch.from_numpy(f["x"]), torch.from_numpy(f["t"])
    np.testing.assert_array_equal(f["x"], W.make_input(21, 2, 1, 64, 64))
    spec = O.param_spec()
    for s in range(3):
        p = f"s{s}_"
        r = O.train_step(P, B, opt, x, t, w_bce=1.0, w_dice=0.0, w_focal=1.0)
        ref = f[p + "logits"]
        assert np.max(np.abs(r["logits"].numpy() - ref)) <= 1e-5 * np.max(np.abs(ref))
        for k in ("bce", "dice", "focal", "loss"):
            assert abs(r[k].item() - float(f[p + k])) < 1e-6, k
        _check_grads(_grad_stats(r["grads"], spec), f[p + "grad_norm"], f[p + "grad_sum"],
                     f[p + "grad_samp"], rtol=1e-4)
        psamp = np.stack([P[it[0]].reshape(-1)[torch.from_numpy(
            np.floor(W.uniform(7, 3000 + ti, 64) * P[it[0]].numel()).astype(np.int64))].numpy()
            for ti, it in enumerate(spec)])
        np.testing.assert_allclose(psamp, f[p + "params_samp"], rtol=0, atol=1e-7)


@pytest.mark.parametrize("tag,B,seed", [("eq_", 4, 22), ("uneq_", 3, 23)])
def test_oracle_dataparallel_focal(golden_dir, tag, B, seed):
    """nn.DataParallel with FocalTversky: loss of the gathered logits (global TP/FP/FN),
    equal shards and DataParallel's unequal chunked scatter (3 -> 2 + 1)."""
    f = _load(golden_dir, "unet_dpf_64.npz")
    wb, wd, wf = (float(v) for v in f[tag + "ratios"])
    P = O.make_params(42)
    x = torch.from_numpy(W.make_input(seed, B, 1, 64, 64))
    t = torch.from_numpy(W.make_target(seed, B, 64, 64))
    r = O.train_step(P, O.init_buffers(), None, x, t, w_bce=wb, w_dice=wd, w_focal=wf, shards=2)
    for k in ("bce", "dice", "focal", "loss"):
        assert abs(r[k].item() - float(f[tag + k])) < 1e-6, k
    _check_grads(_grad_stats(r["grads"], O.param_spec()), f[tag + "grad_norm"],
                 f[tag + "grad_sum"], f[tag + "grad_samp"], rtol=1e-4)


def test_oracle_mod_narrow_widths(golden_dir):
    """The reference grid's narrow widths (config/config.yaml): mod.py UNet(32, 4) over two
    AdamW steps, UNet(24, 3), UNet(48, 3) and ResUNet(16, 3) one step each."""
    from oracle import mod_ref_cpu as MO
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    f = _load(golden_dir, "mod_narrow_64.npz")
    x = torch.from_numpy(W.make_input(31, 2, 1, 64, 64))
    t = torch.from_numpy(W.make_target(31, 2, 64, 64))
    P = MO.make_params(42, 32, 4)
    B = MO.init_buffers(32, 4)
    opt = O.AdamWState(P, lr=1e-4)
    names = [n for n, _ in MO.bn_layers(32, 4)]
    for s in range(2):
        p = f"b32_s{s}_"
        r = MO.train_step(P, B, opt, x, t, depth=4)
        ref = f[p + "logits"]
        assert np.max(np.abs(r["logits"].numpy() - ref)) <= 1e-5 * np.max(np.abs(ref))
        assert abs(r["loss"].item() - float(f[p + "loss"])) < 1e-6
        _check_grads(_grad_stats(r["grads"], MO.param_spec(1, 1, 32, 4)), f[p + "grad_norm"],
                     f[p + "grad_sum"], f[p + "grad_samp"], rtol=1e-4)
        rm = np.concatenate([B[f"{n}.running_mean"].numpy() for n in names])
        np.testing.assert_allclose(rm, f[p + "running_mean"], rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        ev = MO.make_forward(4)(x, P, B, training=False).numpy()
    assert np.max(np.abs(ev - f["b32_eval_logits"])) <= 1e-5 * np.max(np.abs(f["b32_eval_logits"]))
    for tag, base in (("u24_", 24), ("u48_", 48)):
        r = MO.train_step(MO.make_params(42, base, 3), MO.init_buffers(base, 3), None, x, t, depth=3)
        assert np.max(np.abs(r["logits"].numpy() - f[tag + "logits"])) <= 1e-5 * np.max(np.abs(f[tag + "logits"]))
        assert abs(r["loss"].item() - float(f[tag + "loss"])) < 1e-6
        _check_grads(_grad_stats(r["grads"], MO.param_spec(1, 1, base, 3)), f[tag + "grad_norm"],
                     f[tag + "grad_sum"], f[tag + "grad_samp"], rtol=1e-4)
    r = MO.res_train_step(MO.res_make_params(42, 16, 3), MO.res_init_buffers(16, 3), None, x, t, depth=3)
    assert np.max(np.abs(r["logits"].numpy() - f["r16_logits"])) <= 1e-5 * np.max(np.abs(f["r16_logits"]))
    assert abs(r["loss"].item() - float(f["r16_loss"])) < 1e-6
    _check_grads(_grad_stats(r["grads"], MO.res_param_spec(1, 1, 16, 3)), f["r16_grad_norm"],
                 f["r16_grad_sum"], f["r16_grad_samp"], rtol=1e-4)


@pytest.mark.parametrize("tag,lr", [("lr0_", 0.0), ("lr4_", 1e-4)])
def test_oracle_dataparallel_train_then_eval(golden_dir, tag, lr):
    """The oracle's nn.DataParallel epoch (two steps: shards 2 + 2, then replica 0 alone;
    only replica 0's running statistics kept) and its eval forward reproduce the
    reference-generated unet_dpe_64.npz: running statistics and val / test logits."""
    from data.data_loader import SyntheticSegmentation
    f = np.load(os.path.join(golden_dir, "unet_dpe_64.npz"), allow_pickle=False)

    def stack(seed):
        ds = SyntheticSegmentation(5, 64, seed=seed)
        return (torch.stack([ds[i][0] for i in range(5)]), torch.stack([ds[i][1] for i in range(5)]))
    (xtr, ttr), (xva, _), (xte, _) = stack(4), stack(5), stack(6)
    P = O.make_params(42)
    B = O.init_buffers()
    off = 0
    for name in O.BN_LAYERS:
        c = B[f"{name}.running_mean"].numel()
        B[f"{name}.running_mean"] = torch.from_numpy(f[tag + "init_running_mean"][off:off + c].copy())
        B[f"{name}.running_var"] = torch.from_numpy(f[tag + "init_running_var"][off:off + c].copy())
        off += c
    opt = O.AdamWState(P, lr=lr)
    for sl in (slice(0, 4), slice(4, 5)):
        O.train_step(P, B, opt, xtr[sl], ttr[sl], w_bce=1.0, w_dice=0.0, w_focal=1.0, shards=2)
    rm = np.concatenate([B[f"{n}.running_mean"].numpy() for n in O.BN_LAYERS])
    rv = np.concatenate([B[f"{n}.running_var"].numpy() for n in O.BN_LAYERS])
    np.testing.assert_array_equal(rm, f[tag + "running_mean"])
    np.testing.assert_array_equal(rv, f[tag + "running_var"])
    with torch.no_grad():
        np.testing.assert_array_equal(O.forward(xva, P, B, False).numpy(), f[tag + "val_logits"])
        np.testing.assert_array_equal(O.forward(xte, P, B, False).numpy(), f[tag + "test_logits"])


@pytest.mark.parametrize("tag", ["res_", "mod_"])
def test_oracle_dataparallel_modres(golden_dir, tag):
    """nn.DataParallel emulation (shards 2 + 1, per-replica BN, gathered loss, summed
    gradients, replica 0's buffers) of ResUNet(64, 3) and mod.py UNet(64, 3), two AdamW
    steps then eval, against tests/golden/modres_dp_64.npz from the reference modules."""
    from oracle import mod_ref_cpu as MO
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    f = _load(golden_dir, "modres_dp_64.npz")
    if tag == "res_":
        P, B = MO.res_make_params(42, 64, 3), MO.res_init_buffers(64, 3)
        spec, names = MO.res_param_spec(1, 1, 64, 3), [n for n, _ in MO.res_bn_layers(64, 3)]
        step = lambda o, x_, t_: MO.res_train_step(P, B, o, x_, t_, depth=3, shards=2)  # noqa: E731
        fwd = MO.make_res_forward(3)
    else:
        P, B = MO.make_params(42, 64, 3), MO.init_buffers(64, 3)
        spec, names = MO.param_spec(1, 1, 64, 3), [n for n, _ in MO.bn_layers(64, 3)]
        step = lambda o, x_, t_: MO.train_step(P, B, o, x_, t_, depth=3, shards=2)  # noqa: E731
        fwd = MO.make_forward(3)
    opt = O.AdamWState(P, lr=1e-4)
    x = torch.from_numpy(W.make_input(17, 3, 1, 64, 64))
    t = torch.from_numpy(W.make_target(17, 3, 64, 64))
    for s in range(2):
        p = f"{tag}s{s}_"
        r = step(opt, x, t)
        ref = f[p + "logits"]
        assert np.max(np.abs(r["logits"].numpy() - ref)) <= 1e-5 * np.max(np.abs(ref))
        assert abs(r["loss"].item() - float(f[p + "loss"])) < 1e-6
        _check_grads(_grad_stats(r["grads"], spec), f[p + "grad_norm"], f[p + "grad_sum"],
                     f[p + "grad_samp"], rtol=1e-4)
        rm = np.concatenate([B[f"{n}.running_mean"].numpy() for n in names])
        np.testing.assert_allclose(rm, f[p + "running_mean"], rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        ev = fwd(x, P, B, training=False).numpy()
    assert np.max(np.abs(ev - f[tag + "eval_logits"])) <= 1e-5 * np.max(np.abs(f[tag + "eval_logits"]))
