"""CPU-side checks of the C-ABI library: it loads, exports every symbol the header declares,
and its host logic (parameter table, BN table, buckets, workspace planner) agrees with the
reference layout.  No compute is launched (no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import unet_ref_cpu as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "unet_hip.h")


def _header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(unet_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    import unet_hip
    return unet_hip.load()


@pytest.fixture(scope="module")
def rt():
    from unet_hip.runtime import UNetRuntime
    return UNetRuntime("cuda:0")  # creating a context performs no device work


def test_exports_every_header_symbol(lib):
    from unet_hip import _lib
    fns = _header_functions()
    assert len(fns) >= 20
    for f in fns:
        assert hasattr(lib, f), f"libunet_hip.so does not export {f}"
    assert sorted(_lib.SIGNATURES) == fns, "ctypes signature table out of sync with the header"


def test_param_table_matches_reference_layout(rt):
    spec = O.param_spec()
    assert [p[0] for p in rt.params] == [s[0] for s in spec]
    off = 0
    for (name, shape, o), s in zip(rt.params, spec):
        assert tuple(shape) == tuple(s[1]), name
        assert o == off
        off += int(np.prod(shape))
    assert rt.n_param_floats == off == 31_042_369


def test_bn_table(rt):
    assert [b[0] for b in rt.bn] == O.BN_LAYERS
    assert [b[1] for b in rt.bn] == O.BN_CHANNELS
    assert rt.n_bn_floats == 2 * sum(O.BN_CHANNELS)


def test_buckets_partition_the_arena(rt):
    spans = sorted(rt.buckets)
    pos = 0
    for off, n in spans:
        assert off == pos and n > 0
        pos += n
    assert pos == rt.n_param_floats
    # readiness order: decoder side first (highest offsets first)
    offs = [o for o, _ in rt.buckets]
    assert offs == sorted(offs, reverse=True)


def test_workspace_planner(rt):
    a = rt.workspace_bytes(2, 64, 64, True)
    b = rt.workspace_bytes(2, 64, 64, False)
    c = rt.workspace_bytes(32, 256, 256, True)
    assert b < a < c
    # activations dominate: bs=32 @256^2 needs a few GB, well inside 288 GB HBM
    assert 2e9 < c < 40e9
    from unet_hip._lib import HipError
    with pytest.raises(HipError):
        rt.workspace_bytes(2, 60, 64, True)


def test_debug_views_inside_workspace(rt):
    import torch
    N, H, W = 2, 64, 64
    nb = rt.workspace_bytes(N, H, W, True)
    ws = torch.empty(nb, dtype=torch.uint8)
    for i in range(18):
        v, off = rt.debug_view(ws, N, H, W, True, 0, i)
        assert v.shape[0] * v.shape[1] <= nb // 4
    sc = rt.debug_view(ws, N, H, W, True, 1, 3)
    assert sc.numel() == 128
    # the f32 pooled buffer (view 5) exists only where the max-pool writes it: on the x3 path
    # it writes the next conv's x3 image instead, so the view is refused
    from unet_hip._lib import HipError
    with pytest.raises(HipError):
        rt.debug_view(ws, N, H, W, True, 5, 0)
    try:
        rt.set_option("x3", 0)
        ws0 = torch.empty(rt.workspace_bytes(N, H, W, True), dtype=torch.uint8)
        v, _ = rt.debug_view(ws0, N, H, W, True, 5, 0)
        assert tuple(v.shape) == (N * (H // 2) * (W // 2), 64)
    finally:
        rt.set_option("x3", 1)


def test_no_cpu_fallback():
    import torch
    import unet_hip
    m = unet_hip.UNet(1, 1)
    with pytest.raises(unet_hip.HipUnavailable):
        m(torch.zeros(1, 1, 16, 16))
    with pytest.raises(unet_hip.HipUnavailable):
        unet_hip.seg_losses(torch.zeros(1, 1, 16, 16), torch.zeros(1, 1, 16, 16))


def test_state_dict_keys_match_reference():
    import unet_hip
    m = unet_hip.UNet(1, 1)
    names = [n for n, _ in m.named_parameters()]
    assert names == [s[0] for s in O.param_spec()]
    bufs = [n for n, _ in m.named_buffers()]
    want = []
    for n in O.BN_LAYERS:
        want += [f"{n}.running_mean", f"{n}.running_var", f"{n}.num_batches_tracked"]
    assert bufs == want


def test_init_consumes_rng_like_reference():
    """Same seed -> same initial weights as models/model.py:UNet (checked against the
    reference module only where it is importable, i.e. in the build container)."""
    import torch
    import unet_hip
    ref_dir = "/root/reference"
    if not os.path.isdir(ref_dir):
        pytest.skip("reference not present (GPU box)")
    import importlib.util
    spec = importlib.util.spec_from_file_location("_ref_model", os.path.join(ref_dir, "models", "model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(42)
    a = mod.UNet(1, 1)
    torch.manual_seed(42)
    b = unet_hip.UNet(1, 1)
    for (na, pa), (nb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert na == nb and torch.equal(pa, pb), na


# ---------------------------------------------------------------- models/mod.py:UNet
# 64 / 128 run natively; 16 / 24 / 32 / 48 are the reference grid's narrow widths
# (config/config.yaml), run zero-padded inside the library with torch-layout tables
MOD_CFGS = [(64, 3), (64, 5), (128, 5), (16, 3), (16, 5), (24, 4), (24, 6), (32, 3), (32, 5),
            (48, 4), (48, 6)]


def _mod_rt(base, depth):
    from unet_hip import _lib
    from unet_hip.runtime import UNetRuntime
    return UNetRuntime.get("cuda:0", 1, 1, _lib.VARIANT_MOD, base, depth)


@pytest.mark.parametrize("base,depth", MOD_CFGS)
def test_mod_tables_match_reference_layout(base, depth):
    from oracle import mod_ref_cpu as MO
    rt = _mod_rt(base, depth)
    spec = MO.param_spec(1, 1, base, depth)
    assert [p[0] for p in rt.params] == [s[0] for s in spec]
    off = 0
    for (name, shape, o), s in zip(rt.params, spec):
        assert tuple(shape) == tuple(s[1]), name
        assert o == off
        off += int(np.prod(shape))
    assert rt.n_param_floats == off
    assert [(b[0], b[1]) for b in rt.bn] == MO.bn_layers(base, depth)
    spans = sorted(rt.buckets)
    pos = 0
    for o, n in spans:
        assert o == pos and n > 0
        pos += n
    assert pos == rt.n_param_floats
    offs = [o for o, _ in rt.buckets]
    assert offs == sorted(offs, reverse=True)
    if (base, depth) == (128, 5):
        assert rt.n_param_floats == 497_438_849


def test_mod_config4_workspace():
    rt = _mod_rt(128, 5)
    # BASELINE config 4: 512^2, bs >= 8 fits easily in 288 GB
    b = rt.workspace_bytes(8, 512, 512, True)
    assert 10e9 < b < 120e9
    from unet_hip._lib import HipError
    with pytest.raises(HipError):
        rt.workspace_bytes(2, 48, 48, True)  # not a multiple of 2**5


def test_unsupported_configs_rejected():
    from unet_hip import _lib
    from unet_hip.runtime import UNetRuntime
    for args in [(1, 1, _lib.VARIANT_MOD, 20, 4), (1, 1, _lib.VARIANT_MODEL, 64, 5),
                 (3, 1, _lib.VARIANT_MOD, 64, 4), (1, 1, 7, 64, 4),
                 (1, 1, _lib.VARIANT_MOD, 512, 4), (1, 1, _lib.VARIANT_MOD, 48, 7),
                 (1, 1, _lib.VARIANT_MODEL, 32, 4),
                 (1, 1, _lib.VARIANT_MOD, 48, 4, _lib.MATH_BF16)]:
        with pytest.raises(_lib.HipError):
            UNetRuntime("cuda:0", *args)


def test_mod_state_dict_and_rng_like_reference():
    import torch
    import unet_hip
    from oracle import mod_ref_cpu as MO
    m = unet_hip.ModUNet(1, 1, base_filters=64, depth=3)
    assert [n for n, _ in m.named_parameters()] == [s[0] for s in MO.param_spec(1, 1, 64, 3)]
    want = []
    for n, _ in MO.bn_layers(64, 3):
        want += [f"{n}.running_mean", f"{n}.running_var", f"{n}.num_batches_tracked"]
    assert [n for n, _ in m.named_buffers()] == want
    ref_dir = "/root/reference"
    if not os.path.isdir(ref_dir):
        pytest.skip("reference not present (GPU box)")
    import importlib.util
    spec = importlib.util.spec_from_file_location("_ref_mod", os.path.join(ref_dir, "models", "mod.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(42)
    a = mod.UNet(1, 1, base_filters=64, depth=3)
    torch.manual_seed(42)
    b = unet_hip.ModUNet(1, 1, base_filters=64, depth=3)
    for (na, pa), (nb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert na == nb and torch.equal(pa, pb), na


def test_bf16_math_only_for_mod_variant():
    from unet_hip import _lib
    from unet_hip.runtime import UNetRuntime
    with pytest.raises(_lib.HipError):
        UNetRuntime("cuda:0", 1, 1, _lib.VARIANT_MODEL, 0, 0, _lib.MATH_BF16)
    a = UNetRuntime("cuda:0", 1, 1, _lib.VARIANT_MOD, 128, 5, _lib.MATH_BF16)
    b = _mod_rt(128, 5)
    assert a.params == b.params and a.bn == b.bn and a.buckets == b.buckets


@pytest.mark.parametrize("base,depth", [(16, 4), (24, 3), (48, 5)])
def test_res_narrow_tables(base, depth):
    from unet_hip import _lib
    from unet_hip.runtime import UNetRuntime
    from oracle import mod_ref_cpu as MO
    rt = UNetRuntime.get("cuda:0", 1, 1, _lib.VARIANT_RES, base, depth)
    spec = MO.res_param_spec(1, 1, base, depth)
    assert [(p[0], tuple(p[1])) for p in rt.params] == [(s[0], tuple(s[1])) for s in spec]
    assert [(b[0], b[1]) for b in rt.bn] == MO.res_bn_layers(base, depth)
    assert rt.n_param_floats == sum(int(np.prod(s[1])) for s in spec)
    assert rt.workspace_bytes(2, 64, 64, True) > 0


def test_res_tables_and_rng_like_reference():
    import torch
    import unet_hip
    from unet_hip import _lib
    from unet_hip.runtime import UNetRuntime
    from oracle import mod_ref_cpu as MO
    rt = UNetRuntime.get("cuda:0", 1, 1, _lib.VARIANT_RES, 64, 3)
    spec = MO.res_param_spec(1, 1, 64, 3)
    assert [p[0] for p in rt.params] == [s[0] for s in spec]
    assert [tuple(p[1]) for p in rt.params] == [tuple(s[1]) for s in spec]
    assert [(b[0], b[1]) for b in rt.bn] == MO.res_bn_layers(64, 3)
    spans = sorted(rt.buckets)
    pos = 0
    for o, n in spans:
        assert o == pos and n > 0
        pos += n
    assert pos == rt.n_param_floats
    m = unet_hip.ResUNet(1, 1, base_filters=64, depth=3)
    assert [n for n, _ in m.named_parameters()] == [s[0] for s in spec]
    assert rt.workspace_bytes(2, 64, 64, True) > 0
    ref_dir = "/root/reference"
    if not os.path.isdir(ref_dir):
        pytest.skip("reference not present (GPU box)")
    import importlib.util
    sp = importlib.util.spec_from_file_location("_ref_mod2", os.path.join(ref_dir, "models", "mod.py"))
    mod = importlib.util.module_from_spec(sp)
    sp.loader.exec_module(mod)
    torch.manual_seed(42)
    a = mod.ResUNet(1, 1, base_filters=64, depth=3)
    torch.manual_seed(42)
    b = unet_hip.ResUNet(1, 1, base_filters=64, depth=3)
    for (na, pa), (nb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert na == nb and torch.equal(pa, pb), na


def test_schedule_options_are_explicit(rt, monkeypatch):
    """Kernel-schedule options live in the context (unet_set_option), never in the
    environment: a stray UNET_* variable must not change the defaults."""
    from unet_hip._lib import HipError
    from unet_hip.runtime import UNetRuntime
    monkeypatch.setenv("UNET_RG16_TILE", "3")
    monkeypatch.setenv("UNET_DZ_IN_WGRAD", "0")
    fresh = UNetRuntime("cuda:0")
    assert fresh.get_option("rg16_tile") == -1
    assert fresh.get_option("dz_in_wgrad") == 256
    fresh.set_option("dz_in_wgrad", 0)
    assert fresh.get_option("dz_in_wgrad") == 0
    assert rt.get_option("dz_in_wgrad") == 256  # per context
    with pytest.raises(HipError):
        fresh.set_option("no_such_option", 1)
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib_path()], capture_output=True, text=True)
    assert out.returncode == 0 and " getenv" not in out.stdout, "the library reads the environment"


def test_schedule_option_defaults():
    """The measured defaults documented in INTEGRATION.md §3: the pipelined
    row GEMMs (-1 = pick_tile: 18), the three-block 128x64 tiles for the N = 64 / ConvT
    dgrads, the row3 weight gradients with the 128x64 tile on the wide layers, the bf16
    LDS-DMA kernels with the tap-row halo tile, XCD-contiguous tiles."""
    from unet_hip.runtime import UNetRuntime
    fresh = UNetRuntime("cuda:0")
    want = {"tile_n128": -1, "tile_n128_dgrad": -1, "tile_n64": 19, "tile_n64_dgrad": 25,
            "tile_n32": 15, "tile_convt64": 1, "wgrad_row3": 1, "wgrad_row3_big": 21,
            "wgrad_row3_blocks": 1536, "wgrad_blocks": 2048, "rg16": 1, "rg16_tile": -1,
            "rg16_bn_k": 0, "wg16": 1, "wg16_tile": 2, "wgrad16_blocks": 1536,
            "xcd_remap": 1, "xcd16": 1, "tile_convt": -1, "tile_convt_dgrad": 26,
            "dz_in_wgrad": 256, "rg16_r3": 1, "rg16_n128": 20, "rg16_n128_bn": 0, "wg16_r3": 7,
            "convt16": 1, "x3": 1, "x3_tile": -1, "x3_wtile": -1, "x3_wblocks": 1536, "x3_n64": 2, "x3_r3": 1, "x3_wwaves": 3, "x3_wwaves1": 3, "head_fuse": 1, "pool_fuse": 1, "tile_group": 1}
    got = {k: fresh.get_option(k) for k in want}
    assert got == want


def test_header_option_list_matches_library():
    """include/unet_hip.h names every option the library accepts, in OPTION_TABLE order
    (the header list had drifted), and each one round-trips through
    unet_get_option."""
    import re
    from unet_hip import _lib
    from unet_hip.runtime import UNetRuntime
    text = open(_lib.HEADER).read()
    block = text[text.index("Names (runtime.hip OPTION_TABLE"):text.index("Set them between steps")]
    block = block.split("\n", 1)[1]
    header = re.findall(r"[a-z][a-z0-9_]+", block.replace("*", " "))
    lib_names = _lib.option_names()
    assert header == lib_names, (set(header) ^ set(lib_names))
    fresh = UNetRuntime("cuda:0")
    for n in lib_names:
        fresh.get_option(n)


def test_abi_exports_bucket_event():
    """SURVEY §8b's per-bucket readiness event for non-torch RCCL callers is exported."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _lib_path()], capture_output=True, text=True)
    assert " unet_bucket_event" in out.stdout and " unet_option_name" in out.stdout


def _lib_path():
    from unet_hip import _lib
    return _lib.LIB_PATH


def test_flop_counts_agree_with_oracle():
    from oracle import mod_ref_cpu as MO
    from unet_hip.flops import train_flops_per_image
    assert train_flops_per_image(256, 256) == O.train_flops_per_image(256, 256) == 288_475_840_512
    assert train_flops_per_image(512, 512, 128, 5) == MO.train_flops_per_image(512, 512, 128, 5)
    for H, W, base, depth in ((64, 96, 32, 4), (128, 128, 16, 6), (96, 64, 48, 3)):
        assert train_flops_per_image(H, W, base, depth) == MO.train_flops_per_image(H, W, base, depth)


def test_res_flop_count_matches_torch_counter():
    """bench.py --config res prices ResUNet's step with unet_hip.flops (3x3 / ConvT / head
    + the 1x1 skips): its forward part equals torch's own FLOP counter over the oracle's
    ResUNet forward (models/mod.py:86-131)."""
    import torch
    from torch.utils.flop_counter import FlopCounterMode
    from oracle import mod_ref_cpu as MO
    from unet_hip.flops import res_skip_macs, unet_level_macs
    for base, depth, side in ((16, 3, 64), (8, 5, 64)):
        P, B = MO.res_make_params(1, base, depth), MO.res_init_buffers(base, depth)
        with FlopCounterMode(display=False) as fc:
            MO.make_res_forward(depth)(torch.rand(1, 1, side, side), P, B, True)
        want = 2 * (unet_level_macs(side, side, 1, 1, base, depth) + res_skip_macs(side, side, 1, base, depth))
        assert fc.get_total_flops() == want


def test_x3_split_restatement_is_exact_at_the_range_edges():
    """tests/x3_split_ref.py (the restatement of csrc/x3_split.h): h + m + l == v exactly for
    normal and huge finite v (|v| >= 0x1.FFp127 would round to inf in bf16: h takes the
    largest finite bf16 instead), +-inf and NaN keep h = v with m = l = 0, and values with
    subnormal pieces lose at most 2^-134 (bf16's subnormal quantum is 2^-133)."""
    import numpy as np
    import x3_split_ref as X
    v = X.edge_values()
    h, m, lo = X.split(v)
    hf, mf, lf = (X.bf16_to_f32(b).astype(np.float64) for b in (h, m, lo))
    fin = np.isfinite(v)
    s = hf + mf + lf
    exact = fin & (np.abs(v) >= np.ldexp(1.0, -110))
    assert np.all(s[exact] == v[exact].astype(np.float64))
    assert np.all(np.abs(s[fin] - v[fin].astype(np.float64)) <= np.ldexp(1.0, -134))
    assert np.all(np.isfinite(hf[fin])) and np.all(np.isfinite(mf[fin])) and np.all(np.isfinite(lf[fin]))
    inf = np.isinf(v)
    assert np.all(hf[inf] == v[inf]) and np.all(m[inf] == 0) and np.all(lo[inf] == 0)
    nan = np.isnan(v)
    assert nan.any() and np.all(np.isnan(hf[nan])) and np.all(m[nan] == 0) and np.all(lo[nan] == 0)
    huge = fin & (np.abs(v) >= X.BF16_OVF)
    assert huge.sum() >= 6 and np.all(np.abs(hf[huge]) == float(X.BF16_MAX))


def test_x3_split_host_hook_matches_restatement():
    """unet_x3_split_host runs csrc/x3_split.h (the source the device passes use) on the host;
    its bits equal the NumPy restatement everywhere, the edges included."""
    import ctypes
    import numpy as np
    import x3_split_ref as X
    from unet_hip import _lib
    lib = _lib.load()
    v = np.ascontiguousarray(X.edge_values(1))
    out = np.zeros(3 * v.size, np.uint16)
    assert lib.unet_x3_split_host(v.ctypes.data_as(ctypes.c_void_p), v.size,
                                  out.ctypes.data_as(ctypes.c_void_p)) == 0
    want = X.to_image(*X.split(v))
    assert np.array_equal(out, want), np.flatnonzero(out != want)[:8]
    assert lib.unet_x3_split_host(v.ctypes.data_as(ctypes.c_void_p), 31,
                                  out.ctypes.data_as(ctypes.c_void_p)) == -1


def test_backward_refuses_without_a_training_forward(rt):
    """the workspace plan depends on the schedule options, so unet_backward checks
    them against the last training forward's; with no training forward on the context it
    refuses before touching the device."""
    import ctypes
    from unet_hip import _lib
    from unet_hip.runtime import UNetRuntime
    fresh = UNetRuntime("cuda:0")
    d = ctypes.c_void_p(256)
    rc = fresh.lib.unet_backward(fresh.ctx, d, d, d, d, 1 << 30, 2, 64, 64, None)
    assert rc == -1
    assert b"without a training forward" in fresh.lib.unet_last_error(fresh.ctx)
