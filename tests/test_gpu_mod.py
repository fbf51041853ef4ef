"""GPU parity of the models/mod.py UNet variant (bias-free Conv ->
BN -> ReLU blocks, concat [skip, up], configurable base / depth) against the CPU oracle
(oracle/mod_ref_cpu.py) and the reference-generated fixtures (tests/golden/mod_*.npz).

Same bars as tests/test_gpu_parity.py: logits max|d| <= 1e-4 max|ref|, losses <= 1e-5,
gradients <= 1e-2 norm-relative per tensor at step 0."""
import os

import numpy as np
import pytest
import torch

from _helpers import (check_eval, options, grad_errors, hip_mod_model, inputs, masks_agree, norm_rel,
                      rel_max, strict_resync_steps)
from oracle import mod_ref_cpu as MO
from oracle import weights as Wt

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
LOGIT_TOL = 1e-4
GRAD_TOL = 1e-2


@pytest.fixture(autouse=True, scope="module")
def _threads():
    torch.set_num_threads(min(16, os.cpu_count() or 1))


def _golden(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def _step(m, opt, x, t):
    import unet_hip
    opt.zero_grad()
    logits = m(x)
    losses = unet_hip.seg_losses(logits, t)
    loss = losses[0] + losses[1]
    loss.backward()
    opt.step()
    return logits.detach(), losses.detach()


def _check_grad_stats(m, spec, norms, samp, tol, tag):
    named = dict(m.named_parameters())
    for ti, item in enumerate(spec):
        g = named[item[0]].grad.detach().double().cpu().reshape(-1)
        idx = np.floor(Wt.uniform(7, 3000 + ti, 64) * g.numel()).astype(np.int64)
        assert abs(g.norm().item() - norms[ti]) <= tol * norms[ti], f"{tag} {item[0]} norm"
        assert np.max(np.abs(g[idx].numpy() - samp[ti])) <= tol * norms[ti], f"{tag} {item[0]}"


def test_mod_forward_layers_match_oracle():
    """Train-mode forward of UNet(base 64, depth 3), B=2 64x64, logits vs the oracle."""
    P = MO.make_params(42, 64, 3)
    x, _ = inputs(1, 2, 64, 64)
    ref = MO.make_forward(3)(x, P, MO.init_buffers(64, 3), True)
    m = hip_mod_model(P, DEV, 64, 3)
    with torch.no_grad():
        lg = m(x.to(DEV)).cpu()
    assert rel_max(lg.numpy(), ref.numpy()) <= LOGIT_TOL


@pytest.mark.parametrize("tag,seed,lo,hi", [("", 42, 0.5, 1.5), ("neg_", 5, -1.0, 1.0)])
def test_mod_train_steps_match_golden(golden_dir, tag, seed, lo, hi):
    """Two AdamW steps (lr 1e-4) of UNet(base 64, depth 3) vs the reference's own outputs;
    the gamma in [-1, 1] case exercises the max-pool / ReLU masks after a sign flip."""
    import unet_hip
    f = _golden(golden_dir, "mod_d3_64.npz")
    m = hip_mod_model(MO.make_params(seed, 64, 3, lo, hi), DEV, 64, 3)
    opt = unet_hip.HipAdamW(m.parameters(), lr=1e-4)
    x = torch.from_numpy(Wt.make_input(11, 2, 1, 64, 64)).to(DEV)
    t = torch.from_numpy(Wt.make_target(11, 2, 64, 64)).to(DEV)
    spec = MO.param_spec(1, 1, 64, 3)
    names = [n for n, _ in MO.bn_layers(64, 3)]
    for s in range(2):
        p = f"{tag}s{s}_"
        tol = LOGIT_TOL if s == 0 else 2e-3
        logits, losses = _step(m, opt, x, t)
        ref = f[p + "logits"]
        assert rel_max(logits.cpu().numpy(), ref) <= tol, f"{p} logits"
        ok, nd = masks_agree((torch.sigmoid(logits) > 0.5).cpu().numpy().astype(np.uint8),
                             f[p + "mask"], ref, 10 * tol * np.abs(ref).max())
        assert ok, f"{p}: {nd} mask bits differ away from the decision boundary"
        assert abs(losses[0].item() - float(f[p + "bce"])) <= (1e-5 if s == 0 else 1e-4)
        assert abs(losses[1].item() - float(f[p + "dice"])) <= (1e-5 if s == 0 else 1e-4)
        _check_grad_stats(m, spec, f[p + "grad_norm"], f[p + "grad_samp"],
                          GRAD_TOL if s == 0 else 10 * GRAD_TOL, p)
        sd = m.state_dict()
        rm = torch.cat([sd[f"{n}.running_mean"].cpu() for n in names]).numpy()
        btol = 1e-4 if s == 0 else 1e-3
        np.testing.assert_allclose(rm, f[p + "running_mean"], rtol=btol, atol=btol)
    # eval mode (Trainer.validate / test, utils/trainer.py:130,206-250): the oracle resynced
    # from this path's parameters and running statistics, at the north-star bar
    check_eval(m, MO.make_forward(3), x.cpu(), t.cpu())


@pytest.mark.parametrize("seed,lo,hi", [(42, 0.5, 1.5), (5, -1.0, 1.0)])
def test_mod_train_steps_strict_resync(seed, lo, hi):
    """Three AdamW steps (lr 1e-4) of UNet(base 64, depth 3) with the oracle restarted from
    this path's parameters, running statistics and Adam moments at every step: logits at
    1e-4 and gradients within the fp64 envelope at EVERY step (the golden-trajectory test
    above holds steps past 0 only to the 2e-3 trajectory bar, as fp32 noise compounds)."""
    P = MO.make_params(seed, 64, 3, lo, hi)
    x, t = inputs(11, 2, 64, 64)
    m = hip_mod_model(P, DEV, 64, 3)
    strict_resync_steps(m, lambda P_, B_, o, x_, t_: MO.train_step(P_, B_, o, x_, t_, depth=3), x, t)


def test_mod_full_grads_vs_oracle():
    """Every element of every gradient of UNet(base 64, depth 3) vs the oracle."""
    import unet_hip
    P = MO.make_params(42, 64, 3)
    x, t = inputs(3, 2, 64, 64)
    ref = MO.train_step(P, MO.init_buffers(64, 3), None, x, t, depth=3)
    m = hip_mod_model(P, DEV, 64, 3)
    logits = m(x.to(DEV))
    losses = unet_hip.seg_losses(logits, t.to(DEV))
    (losses[0] + losses[1]).backward()
    assert rel_max(logits.detach().cpu().numpy(), ref["logits"].numpy()) <= LOGIT_TOL
    errs = grad_errors(m, ref["grads"])
    worst = max(errs, key=errs.get)
    assert errs[worst] <= GRAD_TOL, f"{worst}: {errs[worst]:.3e}"


def test_mod_config4_architecture(golden_dir):
    """The config-4 network (base 128, depth 5, 497 M params; 2048 / 4096-channel
    bottleneck) at B=2 64x64, one step vs the reference's fixture."""
    import unet_hip
    f = _golden(golden_dir, "mod_c4_64.npz")
    m = hip_mod_model(MO.make_params(42, 128, 5), DEV, 128, 5)
    x = torch.from_numpy(Wt.make_input(12, 2, 1, 64, 64)).to(DEV)
    t = torch.from_numpy(Wt.make_target(12, 2, 64, 64)).to(DEV)
    logits = m(x)
    losses = unet_hip.seg_losses(logits, t)
    (losses[0] + losses[1]).backward()
    assert rel_max(logits.detach().cpu().numpy(), f["logits"]) <= LOGIT_TOL
    assert abs((losses[0] + losses[1]).item() - float(f["loss"])) <= 1e-5
    _check_grad_stats(m, MO.param_spec(1, 1, 128, 5), f["grad_norm"], f["grad_samp"], GRAD_TOL,
                      "c4")


def test_mod_config4_full_size_smoke():
    """Config 4 at its own size (512x512, bs 2): finite loss, and the BN batch statistics
    of the first layer match a torch evaluation of the same conv on the GPU."""
    import unet_hip
    torch.manual_seed(0)
    m = unet_hip.ModUNet(1, 1, base_filters=128, depth=5).to(DEV).train()
    x = torch.rand(2, 1, 512, 512, device=DEV)
    t = (torch.rand(2, 1, 512, 512, device=DEV) > 0.5).float()
    logits = m(x)
    losses = unet_hip.seg_losses(logits, t)
    (losses[0] + losses[1]).backward()
    assert torch.isfinite(logits).all() and torch.isfinite(losses).all()
    g = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    assert torch.isfinite(g).all() and g.abs().sum() > 0
    w = m.encoders[0][0].weight.detach()
    z = torch.nn.functional.conv2d(x, w, None, padding=1)
    bn = m.encoders[0][1]
    mean = z.mean((0, 2, 3))
    # running_mean after one step = 0.1 * batch mean
    assert norm_rel(bn.running_mean.cpu(), 0.1 * mean.cpu()) <= 1e-4


def test_mod_config4_bf16_full_size_vs_f32():
    """Config 4 at 512x512 (bs 2) with bf16 MFMA and the runtime's default per-GEMM tile
    choice (256x256 and 128x128 row GEMMs both occur at this size): two bf16 runs are
    bit-identical, and the logits and gradients stay within bf16 distance of the f32-MFMA
    evaluation of the same step (a gross indexing or pipelining fault in a tile that only
    large M reaches would show as O(1) errors here; the fine parity is the bf16 oracle test
    below at 64x64)."""
    import unet_hip
    torch.manual_seed(0)
    x = torch.rand(2, 1, 512, 512, device=DEV)
    t = (torch.rand(2, 1, 512, 512, device=DEV) > 0.5).float()
    sd0 = None
    outs = []
    for dt in ("fp32", "bf16", "bf16"):
        m = unet_hip.ModUNet(1, 1, base_filters=128, depth=5, mfma_dtype=dt)
        if sd0 is None:
            sd0 = {k: v.clone() for k, v in m.state_dict().items()}
        m.load_state_dict(sd0)
        m = m.to(DEV).train()
        logits = m(x)
        losses = unet_hip.seg_losses(logits, t)
        (losses[0] + losses[1]).backward()
        torch.cuda.synchronize()
        outs.append((logits.detach().clone(),
                     torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone()))
        del m
    (l32, g32), (l16, g16), (l16b, g16b) = outs
    assert torch.equal(l16, l16b) and torch.equal(g16, g16b)
    el = norm_rel(l16.cpu(), l32.cpu())
    eg = norm_rel(g16.cpu(), g32.cpu())
    print(f"config 4 512x512 bf16 vs f32: logits {el:.2e}, all grads {eg:.2e}")
    assert el <= 5e-2 and eg <= 0.15


# ---------------------------------------------------------------- bf16 MFMA (config 4)
def _to64(d):
    return {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in d.items()}


def _bf16_model(P, base, depth):
    import unet_hip
    m = unet_hip.ModUNet(1, 1, base_filters=base, depth=depth, mfma_dtype="bf16")
    sd = m.state_dict()
    for k, v in P.items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    return m.to(DEV).train()


def _bf16_step(m, x, t):
    import unet_hip
    logits = m(x.to(DEV))
    losses = unet_hip.seg_losses(logits, t.to(DEV))
    (losses[0] + losses[1]).backward()
    torch.cuda.synchronize()
    return (logits.detach().clone(),
            {k: p.grad.detach().clone() for k, p in m.named_parameters()},
            {k: b.detach().clone() for k, b in m.named_buffers()})


def _assert_same(a, b, what):
    assert torch.equal(a[0], b[0]), f"{what}: logits"
    for k, g0 in a[1].items():
        assert torch.equal(g0, b[1][k]), f"{what}: grad {k}"
    for k, b0 in a[2].items():
        assert torch.equal(b0, b[2][k]), f"{what}: buffer {k}"


@pytest.mark.parametrize("tile,wtile", [(0, 0), (0, 2), (2, 2), (4, 2)])
def test_rg16_bit_identical_to_register_staged(tile, wtile):
    """The LDS-DMA bf16 GEMMs (kernels_gemm16.hip, fed by the k_to_bf16 operand images:
    row GEMMs and the transposed-read weight gradients) against the register-staged bf16
    kernels (options rg16 = wg16 = 0) on a base-128 network, where every GEMM but the
    Cin = 1 first conv takes the new path: the same bf16 roundings of the same f32 values,
    the same K order, split-K partition and 128-row BN partial groups, so one training step
    gives bit-identical logits, gradients and BN statistics for every row tile (256-row
    tiles included) and every weight-gradient tile.  The tap-row weight gradient (wg16_r3,
    default 7 since r06) sums K in another order and is pinned to the one-tap kernel here
    (its own test: test_wg16_tap_row_bit_identical)."""
    x, t = inputs(23, 2, 128, 128)
    P = MO.make_params(9, 128, 3)
    outs = []
    for flag in (0, 1):
        m = _bf16_model(P, 128, 3)
        with options(m.flatten_().rt, rg16=flag, wg16=flag, rg16_tile=tile, wg16_tile=wtile,
                     wg16_r3=0):
            outs.append(_bf16_step(m, x, t))
    _assert_same(outs[0], outs[1], f"tile {tile}/{wtile}")


@pytest.mark.parametrize("side", [128, 512])
def test_rg16_tile_choice_is_numerically_invisible(side):
    """BASELINE config 4's network (mod.py UNet(128, 5), bf16 MFMA), bs 2: the row-GEMM tile
    (0 = 128x128, 2 = 256x128, 4 = 256x256, 6 = 512x128, auto = the runtime's per-GEMM
    choice) changes speed only -- one training step is bit-identical across all of them (BN
    partials in fixed 128-row groups, gemm_common.h row_epilogue)."""
    x, t = inputs(29, 2, side, side)
    P = MO.make_params(31, 128, 5)
    outs = {}
    for tile in (0, 2, 4, 6, -1):
        m = _bf16_model(P, 128, 5)
        # the tap-row halo tile (19, the auto choice's 256x256 forward / dgrad since r03) sums
        # K in another order: held to the bf16 envelope by test_rg16_halo_tile_within_bf16_error
        with options(m.flatten_().rt, rg16_tile=tile, rg16_r3=0):
            outs[tile] = _bf16_step(m, x, t)
        del m
    for tile in (2, 4, 6, -1):
        _assert_same(outs[0], outs[tile], f"{side}^2 tile {tile} vs 0")


def test_rg16_tile_group_bit_identical():
    """Option tile_group (r06): BASELINE config 4's network at 512^2, bs 2 -- the 16^2 / 32^2
    levels' 2048- and 4096-output GEMMs (128x128 tiles, 16-32 N tiles) walk their tiles in
    groups of M tiles instead of M-major.  One training step is bit-identical."""
    x, t = inputs(79, 2, 512, 512)
    P = MO.make_params(83, 128, 5)
    outs = {}
    for flag in (0, 1):
        m = _bf16_model(P, 128, 5)
        with options(m.flatten_().rt, tile_group=flag):
            outs[flag] = _bf16_step(m, x, t)
        del m
    _assert_same(outs[0], outs[1], "tile_group")


def test_convt16_pool_and_head_fuse_bit_identical():
    """Options convt16, pool_fuse and head_fuse (default on) in a bf16 training step.  convt16:
    the ConvT forward stores bf16 of its output straight into the decoder conv's kept operand
    image (the same RNE rounding of the same f32 value k_to_bf16 applies) and that conv's prep
    pass converts the skip half only.  pool_fuse (r06 on the bf16 path): each encoder block's
    second conv forms its `do` = mask (dskip + routed dpool) inside its bf16 dz pass from the
    max-pool backward's inputs instead of reading a full-resolution do that maxpool_bwd stored.
    head_fuse (r06 on the bf16 path): the last conv's bf16 dz pass forms its `do` = [fma(y, sc,
    sh) > 0] dl w from the logit gradient, so head_bwd stores none.  BASELINE config 4's
    network, one step at 128^2: each off is bit-identical to all on."""
    x, t = inputs(53, 2, 128, 128)
    P = MO.make_params(59, 128, 5)
    outs = {}
    for flags in ((1, 1, 1), (0, 1, 1), (1, 0, 1), (1, 1, 0)):
        m = _bf16_model(P, 128, 5)
        with options(m.flatten_().rt, convt16=flags[0], pool_fuse=flags[1], head_fuse=flags[2]):
            outs[flags] = _bf16_step(m, x, t)
        del m
    _assert_same(outs[(1, 1, 1)], outs[(0, 1, 1)], "convt16")
    _assert_same(outs[(1, 1, 1)], outs[(1, 0, 1)], "pool_fuse")
    _assert_same(outs[(1, 1, 1)], outs[(1, 1, 0)], "head_fuse")


@pytest.mark.parametrize("side", [256, 128])
def test_wg16_tap_row_bit_identical(side):
    """The tap-row bf16 weight gradient (kernels_gemm16.hip wgrad16_row3_kernel, option wg16_r3
    = 4: the three dx taps of one tap row from one halo of 66 pixel rows) runs the same MFMA
    sequence per weight element as the one-tap kernel (same operands, pixel chunks, k-steps and
    split partition), so one training step of BASELINE config 4's network (256^2: tap-row
    levels W = 256, 128, 64; the rest fall back) is bit-identical.  The default, wg16_r3 = 7
    (r06: the 16x16x32 kernel with the re-read stagger, also at W = 32 / 16 as 2 / 4 halo
    segments per 64-pixel chunk: at 128^2 the levels W = 32, 16), sums 32 instead of 16 exact
    bf16 products per MFMA step: f32 rounding apart from those."""
    x, t = inputs(43, 2, side, side)
    P = MO.make_params(47, 128, 5)
    outs = {}
    for r3 in (0, 4, 7):
        m = _bf16_model(P, 128, 5)
        with options(m.flatten_().rt, wg16_r3=r3):
            outs[r3] = _bf16_step(m, x, t)
        del m
    _assert_same(outs[0], outs[4], "wg16_r3=4 vs one-tap")
    assert torch.equal(outs[7][0], outs[4][0])  # the forward does not change
    for k, g4 in outs[4][1].items():
        g7 = outs[7][1][k]
        assert torch.isfinite(g7).all(), k
        tol = 2e-5 * max(g4.abs().max().item(), 1e-30)
        assert (g7 - g4).abs().max().item() <= tol, (k, (g7 - g4).abs().max().item(), tol)


@pytest.mark.parametrize("halo", [19, 20])
def test_rg16_halo_tile_within_bf16_error(halo):
    """Tiles 19 / 20 (the tap-row halo kernel at 256x256 / 512x128, kernels_gemm16.hip
    rowgemm16_row3_kernel) sum K in
    the order (tap row, channel slice, tap column) instead of the one-tap kernel's (tap,
    channel), so it is not bit-identical to tile 4.  BASELINE config 4's network at 256^2
    (halo levels W = 256 .. 16; the 8x8 bottleneck falls back to the one-tap tile), one
    training step: its distance from tile 4 must stay below the distance of tile 4 itself
    from the fp32-MFMA network (the bf16 rounding error the path already carries), for the
    logits and for every gradient (floor 1e-3 for near-zero BN-bias gradients)."""
    x, t = inputs(37, 1, 256, 256)
    P = MO.make_params(41, 128, 5)
    outs = {}
    for tile in (4, halo):
        m = _bf16_model(P, 128, 5)
        with options(m.flatten_().rt, rg16_tile=tile):
            outs[tile] = _bf16_step(m, x, t)
        del m
    import unet_hip
    m = unet_hip.ModUNet(1, 1, base_filters=128, depth=5)
    sd = m.state_dict()
    for k, v in P.items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    f32 = _bf16_step(m.to(DEV).train(), x, t)
    e_l = rel_max(outs[halo][0].cpu(), outs[4][0].cpu())
    b_l = rel_max(outs[4][0].cpu(), f32[0].cpu())
    print(f"logits: halo vs one-tap {e_l:.3e}, bf16 vs fp32 {b_l:.3e}")
    assert e_l <= b_l, (e_l, b_l)
    worst = []
    for k, g4 in outs[4][1].items():
        e = norm_rel(outs[halo][1][k].cpu(), g4.cpu())
        b = norm_rel(g4.cpu(), f32[1][k].cpu())
        worst.append((e / max(b, 1e-3), k, e, b))
    worst.sort(reverse=True)
    print("worst grads (ratio, name, halo-vs-one-tap, bf16-vs-fp32):", worst[:4])
    assert worst[0][0] <= 1.0, worst[:4]


_BF16_ORACLES = {}


def _bf16_oracles(base, depth):
    """The three oracle evaluations test_mod_bf16_matches_bf16_oracle compares against
    (bf16-operand fp32, bf16-operand fp64, plain fp32), computed once per network: they do
    not depend on the HIP tile under test."""
    key = (base, depth)
    if key not in _BF16_ORACLES:
        P = MO.make_params(42, base, depth)
        x, t = inputs(5, 2, 64, 64)
        _BF16_ORACLES[key] = (
            MO.train_step(P, MO.init_buffers(base, depth), None, x, t, depth=depth, bf16=True),
            MO.train_step(_to64(P), _to64(MO.init_buffers(base, depth)), None, x.double(),
                          t.double(), depth=depth, bf16=True),
            MO.train_step(P, MO.init_buffers(base, depth), None, x, t, depth=depth))
    return _BF16_ORACLES[key]


@pytest.mark.parametrize("base,depth,tile", [(64, 3, "4"), (128, 5, "0"), (128, 5, "2"), (128, 5, "4"),
                                             (128, 5, "19"), (128, 5, "20"), (128, 5, "auto")])
def test_mod_bf16_matches_bf16_oracle(base, depth, tile):
    """mfma_dtype="bf16": one step at B=2 64x64 vs the oracle that rounds exactly the GEMM
    operands the HIP bf16 kernels round (oracle/mod_ref_cpu.py, bf16=True).

    Rounding to bf16 is discontinuous: a 1e-7 difference upstream moves an operand across a
    rounding boundary with probability ~1e-5 per element, and the flips compound through
    BN.  The oracle itself shows it: evaluated in fp32 and in fp64 (same bf16 roundings of
    its own values) it differs by ~6e-3 in the logits and up to ~15 % on small BN-bias
    gradients.  The bar is 2x that spread of the oracle against itself.  tile = the
    LDS-DMA GEMM tile (option rg16_tile; "2" = 256 rows x 8 waves, "4" = 256 x 256), with
    the 256x256 weight-gradient tile on the 256-channel layers; "auto" = the runtime's
    per-GEMM choice (rg16_tile, runtime.hip) and default wgrad tile."""
    import unet_hip
    opts = {} if tile == "auto" else dict(
        rg16_tile=int(tile), wg16_tile=2 if tile in ("4", "19", "20") else 0)
    P = MO.make_params(42, base, depth)
    x, t = inputs(5, 2, 64, 64)
    ref, r64, ref32 = _bf16_oracles(base, depth)
    m = unet_hip.ModUNet(1, 1, base_filters=base, depth=depth, mfma_dtype="bf16")
    sd = m.state_dict()
    for k, v in P.items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    with options(m.flatten_().rt, **opts):
        logits = m(x.to(DEV))
        losses = unet_hip.seg_losses(logits, t.to(DEV))
        (losses[0] + losses[1]).backward()
        torch.cuda.synchronize()
    lg = logits.detach().cpu().numpy()
    spread_l = rel_max(ref["logits"].numpy(), r64["logits"].numpy())
    e_l = rel_max(lg, ref["logits"].numpy())
    e_l32 = rel_max(lg, ref32["logits"].numpy())
    spread = {k: norm_rel(ref["grads"][k], r64["grads"][k]) for k in ref["grads"]}
    errs = grad_errors(m, ref["grads"])
    worst = max(errs, key=errs.get)
    env = 2 * max(spread.values())
    print(f"bf16 base {base} depth {depth}: logits vs bf16 oracle {e_l:.2e} (oracle spread "
          f"{spread_l:.2e}), vs fp32 oracle {e_l32:.2e}; worst grad {worst} {errs[worst]:.2e} "
          f"(envelope {env:.2e})")
    assert e_l <= 2 * spread_l + 1e-4
    assert abs((losses[0] + losses[1]).item() - ref["loss"].item()) <= 1e-3
    assert errs[worst] <= env, f"{worst}: {errs[worst]:.3e}"
    # and bf16 stays a bf16-sized perturbation of the fp32 network
    assert e_l32 <= 5e-2


# ---------------------------------------------------------------- narrow widths (padded)
def test_mod_narrow_b32_matches_golden(golden_dir):
    """The reference grid's narrow widths (config/config.yaml: base_filters 16 / 24 / 32 /
    48): mod.py UNet(base 32, depth 4) runs with every level zero-padded to 64 / 128 / ...
    inside the library.  Two AdamW steps vs the reference's own outputs
    (tests/golden/mod_narrow_64.npz) at the usual bars, the running statistics, and the
    eval-mode path from the resynced state."""
    import unet_hip
    f = _golden(golden_dir, "mod_narrow_64.npz")
    m = hip_mod_model(MO.make_params(42, 32, 4), DEV, 32, 4)
    opt = unet_hip.HipAdamW(m.parameters(), lr=1e-4)
    x = torch.from_numpy(Wt.make_input(31, 2, 1, 64, 64)).to(DEV)
    t = torch.from_numpy(Wt.make_target(31, 2, 64, 64)).to(DEV)
    spec = MO.param_spec(1, 1, 32, 4)
    names = [n for n, _ in MO.bn_layers(32, 4)]
    for s in range(2):
        p = f"b32_s{s}_"
        tol = LOGIT_TOL if s == 0 else 2e-3
        logits, losses = _step(m, opt, x, t)
        assert rel_max(logits.cpu().numpy(), f[p + "logits"]) <= tol, f"{p} logits"
        assert abs((losses[0] + losses[1]).item() - float(f[p + "loss"])) <= (1e-5 if s == 0 else 1e-4)
        _check_grad_stats(m, spec, f[p + "grad_norm"], f[p + "grad_samp"],
                          GRAD_TOL if s == 0 else 10 * GRAD_TOL, p)
        sd = m.state_dict()
        rm = torch.cat([sd[f"{n}.running_mean"].cpu() for n in names]).numpy()
        rv = torch.cat([sd[f"{n}.running_var"].cpu() for n in names]).numpy()
        btol = 1e-4 if s == 0 else 1e-3
        np.testing.assert_allclose(rm, f[p + "running_mean"], rtol=btol, atol=btol)
        np.testing.assert_allclose(rv, f[p + "running_var"], rtol=btol, atol=btol)
    check_eval(m, MO.make_forward(4), x.cpu(), t.cpu())


@pytest.mark.parametrize("tag,base", [("u24_", 24), ("u48_", 48)])
def test_mod_narrow_one_step_matches_golden(golden_dir, tag, base):
    import unet_hip
    f = _golden(golden_dir, "mod_narrow_64.npz")
    m = hip_mod_model(MO.make_params(42, base, 3), DEV, base, 3)
    x = torch.from_numpy(Wt.make_input(31, 2, 1, 64, 64)).to(DEV)
    t = torch.from_numpy(Wt.make_target(31, 2, 64, 64)).to(DEV)
    logits = m(x)
    losses = unet_hip.seg_losses(logits, t)
    (losses[0] + losses[1]).backward()
    assert rel_max(logits.detach().cpu().numpy(), f[tag + "logits"]) <= LOGIT_TOL
    assert abs((losses[0] + losses[1]).item() - float(f[tag + "loss"])) <= 1e-5
    _check_grad_stats(m, MO.param_spec(1, 1, base, 3), f[tag + "grad_norm"], f[tag + "grad_samp"],
                      GRAD_TOL, tag)


@pytest.mark.parametrize("base,depth,H,W", [(16, 5, 64, 96), (24, 4, 128, 64), (48, 6, 128, 256),
                                            (32, 4, 64, 64)])
def test_mod_narrow_full_grads_vs_fp64(base, depth, H, W):
    """Every gradient element of narrow networks (base 32 native on the 32-channel tiles;
    16 / 24 padded to 32 and 48 to 64 inside the library) against the
    fp64 oracle, and the padding is invisible in the caller's arenas (torch-layout
    gradients, running stats).  At depth 6 the bottleneck BN sees 16 values per channel,
    where a near-zero ReLU input flips under any fp32 rounding change: the envelope is 2x
    the fp32 oracle's own error over x and x * (1 + 1e-7) (as tests/test_gpu_res.py),
    floor 1e-2."""
    import unet_hip
    from _helpers import options
    P = MO.make_params(7, base, depth)
    x, t = inputs(33, 2, H, W)
    ref = MO.train_step(P, MO.init_buffers(base, depth), None, x, t, depth=depth)
    refp = MO.train_step(P, MO.init_buffers(base, depth), None, x * (1 + 1e-7), t, depth=depth)
    r64 = MO.train_step({k: v.double() for k, v in P.items()},
                        {k: (v.double() if v.is_floating_point() else v.clone())
                         for k, v in MO.init_buffers(base, depth).items()},
                        None, x.double(), t.double(), depth=depth)
    m = hip_mod_model(P, DEV, base, depth)
    with options(m.flatten_().rt):
        logits = m(x.to(DEV))
        losses = unet_hip.seg_losses(logits, t.to(DEV))
        (losses[0] + losses[1]).backward()
    assert rel_max(logits.detach().cpu().numpy(), ref["logits"].numpy()) <= LOGIT_TOL
    e32 = {k: max(norm_rel(g, r64["grads"][k]), norm_rel(refp["grads"][k], r64["grads"][k]))
           for k, g in ref["grads"].items()}
    env = max(2 * max(e32.values()), GRAD_TOL)
    errs = grad_errors(m, r64["grads"])
    worst = max(errs, key=errs.get)
    assert errs[worst] <= env, f"{worst}: {errs[worst]:.3e} (fp32 oracle {e32[worst]:.3e})"
    Bref = MO.init_buffers(base, depth)
    MO.make_forward(depth)(x, P, Bref, True)
    for k, v in m.named_buffers():
        if v.is_floating_point():
            np.testing.assert_allclose(v.cpu().numpy(), Bref[k].numpy(), rtol=1e-4, atol=1e-5, err_msg=k)
