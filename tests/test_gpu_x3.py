"""f32 GEMMs on the bf16 matrix cores through exact three-way operand splits (option x3,
csrc/kernels_gemm_x3.hip) against the f32-MFMA kernels (option x3 = 0), both measured
against the oracle evaluated in fp64.

Every f32 operand splits exactly into three bf16 pieces (csrc/x3_split.h); the kernels form
six of the nine piece products (the three dropped ones are at most ~2^-23 |a b| together) and
keep the five small products in a separate f32 accumulator, so the large accumulator takes one
rounding per 16 products against the f32 MFMA's one per 2.  Bars: "no worse than the f32 MFMA
path" per layer and on the logits, plus ABSOLUTE bars against an fp64 oracle that follows the
GPU's own branches (oracle/unet_ref_cpu.py relu_masks / pool_idx: a pre-activation within ~1e-6
of zero rounds to the other side in one f32 evaluation or another, and a near-tie of two BN
outputs in a max-pool window routes the gradient to another pixel; either moves whole upstream
gradients, which is what the relative bars used to absorb).  The 1e-4 north-star bars are the
other GPU tests' (they run the default, x3 on).
"""
import os

import numpy as np
import pytest
import torch

from _helpers import hip_model, inputs, norm_rel
from oracle import unet_ref_cpu as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(autouse=True, scope="module")
def _threads():
    torch.set_num_threads(min(16, os.cpu_count() or 1))


def _to64(d):
    return {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in d.items()}


# Absolute bars against the fp64 oracle on the GPU's own ReLU / max-pool branches (measured r05
# on MI355X, profiles/r05_x3_masked_bars.txt: worst weight gradient 4.9e-6 (x3) / 1.3e-5 (f32
# MFMA) at 128^2, 1.3e-5 / 1.4e-5 (halo / one-tap x3) at 256^2; worst bias / BN gradient
# 6.1e-6 .. 2.4e-5).  The conv biases ahead of ReLU -> BN (models/model.py:36-38) get sums that
# largely cancel (the BN input gradient sums to ~0 over the pixels), so their relative rounding
# noise is the larger; every tensor is also held to SURVEY §8c's 1e-2.
W_BAR, B_BAR, ALL_BAR = 1e-4, 2e-4, 1e-2


def _relu_masks(m, x):
    """The 18 conv ReLU decisions (y > 0, NCHW) and the 4 max-pool winner indices of this
    path's training forward on x (the forward is deterministic, so they are the ones m(x)
    takes)."""
    st = m.flatten_()
    N, _, H, W = x.shape
    with torch.no_grad():
        _, ws = st.rt.forward(st.param_arena, st.bn_arena.clone(), st.nbt_arena.clone(),
                              x.to(DEV), training=True)
    masks = []
    for i in range(18):
        v, off = st.rt.debug_view(ws, N, H, W, True, 0, i)
        lvl = {0: 0, 1: 0, 2: 1, 3: 1, 4: 2, 5: 2, 6: 3, 7: 3, 8: 4, 9: 4, 10: 3, 11: 3,
               12: 2, 13: 2, 14: 1, 15: 1, 16: 0, 17: 0}[i]
        C = 64 << lvl
        h, w = H >> lvl, W >> lvl
        masks.append((v[:, off:off + C] > 0).reshape(N, h, w, C).permute(0, 3, 1, 2).cpu())
    pools = []
    for lvl in range(4):
        v, _ = st.rt.debug_view(ws, N, H, W, True, 8, lvl)
        C, h, w = 64 << lvl, H >> (lvl + 1), W >> (lvl + 1)
        pools.append(v.reshape(N, h, w, C).permute(0, 3, 1, 2).cpu())
    del ws
    return masks, pools


def _masked_fp64_step(P, x, t, branches):
    masks, pools = branches
    return O.train_step(_to64(P), _to64(O.init_buffers()), None, x.double(), t.double(),
                        forward_fn=lambda xx, PP, BB, tr: O.forward(xx, PP, BB, tr, relu_masks=masks,
                                                                   pool_idx=pools))


def _check_masked(grads, ref, tag):
    """Per-tensor norm-relative gradient errors against the masked fp64 step: weights <=
    W_BAR, conv / BN biases <= B_BAR, every tensor <= ALL_BAR.  Returns the worst of each."""
    ew = {k: norm_rel(grads[k], g) for k, g in ref["grads"].items() if g.dim() == 4}
    eb = {k: norm_rel(grads[k], g) for k, g in ref["grads"].items() if g.dim() != 4}
    kw, kb = max(ew, key=ew.get), max(eb, key=eb.get)
    print(f"{tag}: vs masked fp64: worst weight {kw} {ew[kw]:.2e}, worst other {kb} {eb[kb]:.2e}")
    assert ew[kw] <= W_BAR, (tag, kw, ew[kw])
    assert max(eb.values()) <= ALL_BAR, (tag, kb, eb[kb])
    assert all(v <= B_BAR for v in eb.values()), (tag, kb, eb[kb])
    return ew[kw], eb[kb]


def test_x3_forward_no_less_accurate_than_f32_mfma():
    """B=2 at 128x128 (every conv but the Cin = 1 first one and every ConvT on x3 kernels):
    each layer's output and the logits, relative to the fp64 oracle, with x3 on and off.
    The x3 error must not exceed the f32 MFMA kernels' by more than 25 % at any layer (in
    practice it is ~3x smaller, profiles/r04_x3_probe_*.txt)."""
    P = O.make_params(7)
    x, _ = inputs(3, 2, 128, 128)
    rec = []
    ref = O.forward(x.double(), _to64(P), _to64(O.init_buffers()), True, record=rec)
    errs = {}
    from _helpers import options
    for x3 in (1, 0):
        m = hip_model(P, DEV)
        st = m.flatten_()
        with options(st.rt, x3=x3), torch.no_grad():
            logits, ws = st.rt.forward(st.param_arena, st.bn_arena, st.nbt_arena, x.to(DEV),
                                       training=True)
            torch.cuda.synchronize()
        e = []
        for i in range(18):
            v, off = st.rt.debug_view(ws, 2, 128, 128, True, 0, i)
            C = rec[i].shape[1]
            got = v[:, off:off + C].cpu().double()
            want = rec[i].permute(0, 2, 3, 1).reshape(-1, C)
            e.append(norm_rel(got, want))
        e.append(norm_rel(logits.cpu().double(), ref))
        errs[x3] = np.array(e)
        del m, st, ws
    print("per-layer norm-rel error vs fp64, x3:", np.array2string(errs[1], precision=2))
    print("per-layer norm-rel error vs fp64, f32:", np.array2string(errs[0], precision=2))
    assert np.all(errs[1] <= 1.25 * errs[0] + 1e-8), (errs[1], errs[0])
    assert errs[1][-1] <= 1e-5


def test_x3_train_step_matches_f32_mfma():
    """One training step (fwd, BCE+Dice, bwd) at B=2 128x128 against the fp64 oracle: logits
    at least as accurate as the f32-MFMA path's (measured 1.2e-6 vs 3.1e-6); gradients against
    the fp64 step that follows each path's own ReLU branches at the absolute bars above, and
    x3's worst tensor no worse than 1.25x the f32 path's on the same footing.  (Against the
    unmasked fp64 step a ReLU input within ~1e-6 of zero flips in one evaluation or the other
    and moves upstream gradients by ~1e-2)"""
    import unet_hip
    P = O.make_params(11)
    x, t = inputs(5, 2, 128, 128)
    ref = O.train_step(_to64(P), _to64(O.init_buffers()), None, x.double(), t.double())
    res, worst = {}, {}
    from _helpers import options
    for x3 in (1, 0):
        m = hip_model(P, DEV)
        with options(m.flatten_().rt, x3=x3):
            masks = _relu_masks(m, x)
            logits = m(x.to(DEV))
            losses = unet_hip.seg_losses(logits, t.to(DEV))
            (losses[0] + losses[1]).backward()
            torch.cuda.synchronize()
        res[x3] = (logits.detach().cpu().double(),
                   {k: p.grad.detach().cpu().double() for k, p in m.named_parameters()})
        del m
        worst[x3] = _check_masked(res[x3][1], _masked_fp64_step(P, x, t, masks), f"x3={x3}")
    el = {k: norm_rel(res[k][0], ref["logits"]) for k in res}
    assert el[1] <= 1e-5 and el[1] <= 1.25 * el[0] + 1e-8, el
    print(f"logits vs fp64: x3 {el[1]:.2e} f32 {el[0]:.2e}")
    assert worst[1][0] <= 1.25 * worst[0][0] + 1e-7, worst


@pytest.mark.parametrize("B,H,W", [(2, 128, 128), (1, 48, 80)])
def test_x3_row_tile_choice_bit_identical(B, H, W):
    """Every one-tap x3 row-GEMM tile (0 = 256x128, 1 = 128x128, 2 = 128x64, 3 = 256x64 for the
    64-output GEMMs; -1 = the per-GEMM choice) walks K in the same chunk order with the same
    six-product MFMA sequence per element and emits BN partials in the same 128-row groups, so
    one training step -- logits and the whole gradient arena -- is bit-identical across them
    (48x80: tiles ending past M, the guarded epilogue)."""
    import unet_hip
    from _helpers import options
    x, t = inputs(13, B, H, W)
    outs = []
    runs = ((-1, 2), (0, 2), (1, 2), (2, 2), (-1, 3))
    for tile, n64 in runs:
        m = hip_model(O.make_params(42), DEV)
        # (the tap-row halo tiles sum K in another order: test_x3_halo_tile_matches_one_tap)
        with options(m.flatten_().rt, x3_tile=tile, x3_n64=n64, x3_r3=0):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        outs.append((logits.detach().clone(), m._state.grad_arena.clone()))
        del m
    for i in range(1, len(outs)):
        assert torch.equal(outs[0][0], outs[i][0]), i
        assert torch.equal(outs[0][1], outs[i][1]), (i, (outs[0][1] - outs[i][1]).abs().max().item())
    assert torch.isfinite(outs[0][1]).all()


@pytest.mark.parametrize("variant", ["model", "mod"])
def test_x3_head_fuse_bit_identical(variant):
    """Options head_fuse / pool_fuse (r05, default on): the x3 dz pass of the last conv
    recomputes its `do` = [activation > 0] dl w from the logit gradient, and that of each
    encoder block's second conv its `do` = mask (dskip + routed dpool) from the max-pool
    backward's inputs (the producers' own fma masks and sums), instead of reading a
    full-resolution f32 `do` the producer stored: one training step is bit-identical.  "mod"
    (ADVICE r05): models/mod.py UNet(64, 3) in f32, whose BN -> ReLU order takes the mask
    branches (the head's fma(y, sc, sh) > 0 and the pool's fma(msc, y, msh) > 0)."""
    import unet_hip
    from _helpers import hip_mod_model, options
    from oracle import mod_ref_cpu as MO
    x, t = inputs(47, 2, 128, 128)
    outs = []
    for flag in (0, 1):
        if variant == "model":
            m = hip_model(O.make_params(53), DEV)
        else:
            m = hip_mod_model(MO.make_params(53, 64, 3), DEV, 64, 3)
        with options(m.flatten_().rt, head_fuse=flag, pool_fuse=flag):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        outs.append((logits.detach().clone(), m._state.grad_arena.clone()))
        del m
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1]), (outs[0][1] - outs[1][1]).abs().max().item()


def test_tile_group_order_bit_identical():
    """Option tile_group (r06, default on): the LDS-DMA row GEMMs walk their tiles in groups of M
    tiles (gemm_common.h tile_mn) where the N tiles are many, so one XCD's resident blocks share
    fewer weight rows.  A tile computes the same thing wherever it runs: one training step of the
    model.py network at 256^2, bs 4 (the 16^2 level's 1024-output GEMMs take groups of 2) is
    bit-identical to the M-major order."""
    import unet_hip
    from _helpers import options
    x, t = inputs(71, 4, 256, 256)
    outs = []
    for flag in (0, 1):
        m = hip_model(O.make_params(73), DEV)
        with options(m.flatten_().rt, tile_group=flag):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        outs.append((logits.detach().clone(), m._state.grad_arena.clone()))
        del m
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1]), (outs[0][1] - outs[1][1]).abs().max().item()


def test_x3_tap_row_wgrad_matches_one_tap():
    """The tap-row x3 weight gradient (wgrad_x3_row3_kernel: three dx taps from one 34-pixel
    halo, default on rows of 32k pixels) against the one-tap x3 kernel (option x3_wtile = 1
    everywhere): the same products summed over other split partitions, so every weight and
    bias gradient agrees to f32 summation noise (<= 1e-5 norm-relative); the forward is
    unchanged (logits bit-identical).  B=2 at 128x128: W = 128, 64, 32 on the tap-row kernel,
    16 and 8 on the one-tap kernel either way."""
    import unet_hip
    from _helpers import options
    x, t = inputs(19, 2, 128, 128)
    outs = []
    for wt in (-1, 1):
        m = hip_model(O.make_params(42), DEV)
        with options(m.flatten_().rt, x3_wtile=wt):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        outs.append((logits.detach().clone(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
        del m
    assert torch.equal(outs[0][0], outs[1][0])
    worst = max(norm_rel(outs[0][1][k].cpu(), g.cpu()) for k, g in outs[1][1].items())
    print(f"tap-row vs one-tap x3 weight gradients: worst norm-rel {worst:.2e}")
    assert worst <= 1e-5


def test_x3_convt_into_decoder_image_bit_identical():
    """Option convt16 on the x3 path: the ConvT forward's epilogue writes the x3 split of its
    output straight into the decoder conv's kept x3 image (the same RNE splits of the same
    f32 values the prep pass forms) and that conv's prep converts the skip half only.  One
    training step at B=2 128x128 is bit-identical to convt16 = 0."""
    import unet_hip
    from _helpers import options
    x, t = inputs(23, 2, 128, 128)
    outs = []
    for flag in (0, 1):
        m = hip_model(O.make_params(42), DEV)
        with options(m.flatten_().rt, convt16=flag):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        outs.append((logits.detach().clone(), m._state.grad_arena.clone()))
        del m
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_x3_halo_tile_no_less_accurate_than_one_tap():
    """The tap-row halo x3 GEMM (rowgemm_x3_row3_kernel, tiles 4 / 5: one 32-channel group of
    one tap row's halo feeds the three dx taps; default on the 3x3 GEMMs of power-of-two
    rows) sums K in (dy, group, dx) instead of the one-tap tiles' (dy, dx, group) order
    (option x3_r3 = 0), so the two agree to f32 rounding, not bitwise -- and the conv biases
    of this network (conv -> bias -> ReLU -> BN, models/model.py:36-38) get gradients that
    largely cancel, whose relative rounding noise reaches ~6e-3 between the two orders.  So
    both are judged against the fp64 oracle, as test_x3_train_step_matches_f32_mfma does:
    B=2 at 256x256 (W = 256 .. 16 on the halo kernel, the 256x64 tile on level 0).  At
    1 x 48 x 80 (W not a power of two) no GEMM takes the halo kernel: bit-identical."""
    import unet_hip
    from _helpers import options
    P = O.make_params(42)

    def step(x, t, r3):
        m = hip_model(P, DEV)
        with options(m.flatten_().rt, x3_r3=r3):
            logits = m(x.to(DEV))
            l = unet_hip.seg_losses(logits, t.to(DEV))
            (l[0] + l[1]).backward()
            torch.cuda.synchronize()
        return (logits.detach().cpu().double(),
                {k: p.grad.detach().cpu().double() for k, p in m.named_parameters()})

    x, t = inputs(29, 2, 256, 256)
    ref = O.train_step(_to64(P), _to64(O.init_buffers()), None, x.double(), t.double())
    res = {r3: step(x, t, r3) for r3 in (1, 0)}
    el = {k: norm_rel(res[k][0], ref["logits"]) for k in res}
    print(f"vs fp64: logits halo {el[1]:.2e} one-tap {el[0]:.2e}")
    assert el[1] <= 1e-5 and el[1] <= 1.25 * el[0] + 1e-8, el
    # gradients: absolute bars against the fp64 step on each schedule's own ReLU branches
    worst = {}
    for r3 in (1, 0):
        m = hip_model(P, DEV)
        with options(m.flatten_().rt, x3_r3=r3):
            masks = _relu_masks(m, x)
        del m
        worst[r3] = _check_masked(res[r3][1], _masked_fp64_step(P, x, t, masks), f"x3_r3={r3}")
    assert worst[1][0] <= 1.25 * worst[0][0] + 1e-7, worst
    x, t = inputs(29, 1, 48, 80)
    a, b = step(x, t, 1), step(x, t, 0)
    assert torch.equal(a[0], b[0]) and all(torch.equal(a[1][k], b[1][k]) for k in a[1])


def test_x3_split_device_matches_restatement():
    """The device split pass (to_x3_kernel through unet_x3_split_device, hardware bf16
    conversion) against the NumPy restatement of csrc/x3_split.h: bit-identical over normal
    values of every exponent, huge finite values around the bf16 overflow threshold (h = the
    largest finite bf16), +-inf (h = v, m = l = 0), subnormal and tiny values, signed zeros;
    NaN keeps a NaN h with m = l = 0."""
    import x3_split_ref as X
    import unet_hip
    m = hip_model(O.make_params(42), DEV)
    rt = m.flatten_().rt
    v = X.edge_values(2)
    vd = torch.from_numpy(v).to(DEV)
    out = torch.zeros(3 * v.size, dtype=torch.int16, device=DEV)
    rc = rt.lib.unet_x3_split_device(rt.ctx, vd.data_ptr(), v.size, out.data_ptr(),
                                     unet_hip._lib.stream_ptr(DEV))
    assert rc == 0
    got = out.cpu().numpy().view(np.uint16)
    want = X.to_image(*X.split(v))
    gh, gm, gl = X.from_image(got)
    wh, wm, wl = X.from_image(want)
    nan = np.isnan(v)
    assert np.array_equal(gm, wm) and np.array_equal(gl, wl)
    assert np.array_equal(gh[~nan], wh[~nan]), np.flatnonzero(gh != wh)[:8]
    assert np.all(np.isnan(X.bf16_to_f32(gh[nan])))


@pytest.mark.parametrize("beta", [3.395e38, -3.4e38, float("nan"), 1e-39, float("inf"), float("-inf")])
def test_x3_range_edge_activation_through_one_conv(beta):
    """An activation at the range edges through one x3 conv: channel 5 of encoder1's first BN
    gets gamma = 0, beta = `beta`, so encoder1.3 (64 -> 64, the halo x3 GEMM) reads that value
    at every pixel, split by the forward's to_x3 pass.  Against the f32 MFMA kernels (x3 = 0)
    on the same input: huge finite values (above bf16's overflow threshold; before r05 their
    split overflowed to inf and turned the conv into NaN), NaN and subnormal values give the
    same outputs (finite ones within 1e-5 norm-relative).  +-inf: h = +-inf, m = l = 0, so an
    output is +-inf or NaN as in f32, except that a weight whose low piece is exactly 0 turns
    an inf product into inf * 0 = NaN (x3_split.h caveat): after the ReLU (NaN -> 0 on both
    paths) such outputs read 0 where f32 has +inf; nothing else may differ."""
    P = O.make_params(42)
    P["encoder1.2.weight"][5] = 0.0
    P["encoder1.2.bias"][5] = beta
    x, _ = inputs(3, 2, 64, 64)
    from _helpers import options
    y = {}
    for x3 in (1, 0):
        m = hip_model(P, DEV)
        st = m.flatten_()
        with options(st.rt, x3=x3), torch.no_grad():
            _, ws = st.rt.forward(st.param_arena, st.bn_arena, st.nbt_arena, x.to(DEV), training=True)
            v, off = st.rt.debug_view(ws, 2, 64, 64, True, 0, 1)
            y[x3] = v[:, off:off + 64].cpu().double()
        del m, st, ws
    a, b = y[1], y[0]
    fa, fb = torch.isfinite(a), torch.isfinite(b)
    if np.isinf(beta):
        diff = ~((a == b) | (torch.isnan(a) & torch.isnan(b)))
        assert torch.all((b[diff] == float("inf")) & (a[diff] == 0)), "x3 differs beyond inf*0"
        assert diff.double().mean() <= 0.1
        return
    assert torch.equal(fa, fb)
    assert torch.equal(torch.isnan(a), torch.isnan(b))
    if fa.any():
        assert norm_rel(a[fa], b[fa]) <= 1e-5, norm_rel(a[fa], b[fa])
    if abs(beta) > 1e38:
        assert fa.all() and a.abs().max() > 1e35  # the huge channel reached the outputs


def test_backward_refuses_options_changed_since_forward():
    """unet_backward checks the schedule options against the training forward's
    (the workspace plan and the saved x3 images depend on x3, convt16, ...): toggling x3
    between the two raises instead of reading saved activations at shifted offsets."""
    from _helpers import options
    from unet_hip._lib import HipError
    m = hip_model(O.make_params(42), DEV)
    st = m.flatten_()
    x, _ = inputs(3, 2, 64, 64)
    grads = torch.zeros_like(st.param_arena)
    logits, ws = st.rt.forward(st.param_arena, st.bn_arena, st.nbt_arena, x.to(DEV), training=True)
    with options(st.rt, x3=0):
        with pytest.raises(HipError, match="x3"):
            st.rt.backward(st.param_arena, torch.ones_like(logits), grads, ws)
    st.rt.backward(st.param_arena, torch.ones_like(logits), grads, ws)  # same options: runs
    torch.cuda.synchronize()
    assert torch.isfinite(grads).all()
