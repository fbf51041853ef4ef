"""Drop-in ``UNet`` modules whose forward/backward run on libunet_hip.so:

* ``UNet``    -- models/model.py:5-73
* ``ModUNet`` -- models/mod.py:9-66 (``UNet(in, out, base_filters, depth)``)
* ``ResUNet`` -- models/mod.py:71-131 (residual blocks; what the reference main.py:122 builds)

Each keeps its reference's exact submodule tree (model.py: encoder1..4, middle,
decoder3..1, final; mod.py: encoders, pools, bottleneck, upconvs, decoders, final_conv;
Conv2d / ReLU / BatchNorm2d / ConvTranspose2d in the same Sequential slots), so

* ``state_dict()`` keys, shapes and torch layouts are identical and checkpoints move
  freely between this module and the reference (``main.py:141-142`` style loading);
* construction consumes the torch RNG exactly like the reference, so ``set_seed(42)``
  (utils/utils.py:47-51) gives the same initial weights.

The submodules are never *executed*: on the first forward on a GPU the parameters and
BN buffers are re-pointed into flat device arenas in the native table's order (one
arena for parameters, one for running_mean|running_var, one int64 vector for
num_batches_tracked) and the whole network runs as one native call.  Moving the module
(``.to()``, ``.cuda()``) re-flattens lazily.  CPU tensors raise ``HipUnavailable``:
there is no silent CPU fallback.
"""
import weakref

import torch
import torch.nn as nn

from . import _lib
from ._lib import HipUnavailable
from .functional import UNetFunction
from .runtime import UNetRuntime


def _conv_block(cin, cout):
    # models/model.py:33-43: Conv3x3(bias) -> ReLU -> BN -> Conv3x3 -> ReLU -> BN
    layers = []
    for a, b in ((cin, cout), (cout, cout)):
        layers += [nn.Conv2d(a, b, kernel_size=3, padding=1), nn.ReLU(inplace=True), nn.BatchNorm2d(b)]
    return nn.Sequential(*layers)


def _upconv_block(cin, cout):
    # models/model.py:45-51
    return nn.Sequential(_conv_block(cin, cin // 2),
                         nn.ConvTranspose2d(cin // 2, cout, kernel_size=2, stride=2))


# parameter arena (data_ptr, numel) -> its _ArenaState, so HipAdamW finds the context whose
# fused AdamW + repack (unet_adamw_repack) knows the arena's layout
_ARENAS = weakref.WeakValueDictionary()


def arena_owner(flat):
    """The _ArenaState whose parameter arena is exactly `flat` (same storage span), or None."""
    st = _ARENAS.get((flat.data_ptr(), flat.numel()))
    if st is None or st.param_arena.data_ptr() != flat.data_ptr():
        return None
    return st


class _ArenaState:
    """Flat device arenas shared by the module and the autograd function."""

    def __init__(self, rt, params, param_arena, bn_arena, nbt_arena):
        self.rt = rt
        self.params = params            # [(Parameter, offset, shape)]
        self.param_arena = param_arena
        self.bn_arena = bn_arena
        self.nbt_arena = nbt_arena
        self.grad_arena = None
        # the torch version counters (the arena's plus every parameter's: a Parameter whose
        # .data was re-pointed into the arena keeps its own counter) when the native weight
        # images were last known to match the parameters: None = never (the first forward
        # repacks).  Any torch in-place write to a parameter (load_state_dict, a torch optimizer,
        # user code under no_grad) bumps one of them; the native AdamW writes through the
        # pointer and bumps none.  Writes through `.data` bypass every counter, as they bypass
        # autograd: call the module's params_changed() after those.
        self.native_version = None
        _ARENAS[(param_arena.data_ptr(), param_arena.numel())] = self
        # a new arena may reuse the address of one whose images the (shared) context holds
        rt.params_changed()

    def version(self):
        return self.param_arena._version + sum(p._version for p, _, _ in self.params)

    def sync_params(self):
        """Tell the native side when the parameters changed outside unet_adamw_repack."""
        v = self.version()
        if v != self.native_version:
            self.rt.params_changed()
            self.native_version = v

    def grad_arena_for_backward(self):
        # gradients are written with '=' semantics (zero_grad(set_to_none) is the reference's
        # pattern, utils/trainer.py:81).  If .grad still aliases the arena (accumulation
        # across backward calls), hand autograd a fresh arena so it can add.
        if self.grad_arena is None:
            self.grad_arena = torch.empty_like(self.param_arena)
            return self.grad_arena
        p0 = self.params[0][0]
        if p0.grad is not None and p0.grad.data_ptr() == self.grad_arena.data_ptr():
            return torch.empty_like(self.param_arena)
        return self.grad_arena

    def grad_views(self, arena):
        return [arena[off:off + p.numel()].view(p.shape) for p, off, _ in self.params]


class _HipUNet(nn.Module):
    """Arena management and the native forward shared by both reference networks."""

    _name = "UNet"

    def _native_cfg(self):
        """(in_channels, out_channels, variant, base_filters, depth, math) of the native graph."""
        raise NotImplementedError

    # ---------------------------------------------------------------- arenas
    def _bn_modules(self):
        return {n: m for n, m in self.named_modules() if isinstance(m, nn.BatchNorm2d)}

    def _arenas_valid(self, rt):
        st = self._state
        if st is None or st.rt is not rt:
            return False
        base = st.param_arena.data_ptr()
        for p, off, _ in st.params:
            if p.data_ptr() != base + 4 * off or not p.is_contiguous() or p.device != st.param_arena.device:
                return False
        bns = self._bn_modules()
        bbase = st.bn_arena.data_ptr()
        for name, ch, off in rt.bn:
            if bns[name].running_mean.data_ptr() != bbase + 4 * off:
                return False
        return True

    def flatten_(self):
        """Re-point parameters and BN buffers into flat device arenas (idempotent)."""
        p0 = next(self.parameters())
        dev = p0.device
        if dev.type != "cuda":
            raise HipUnavailable(f"{self._name} runs on the MI355X HIP path only; move it to a "
                                 "GPU with .cuda() / .to('cuda') (no CPU fallback)")
        rt = UNetRuntime.get(dev, *self._native_cfg())
        if self._arenas_valid(rt):
            return self._state
        named = dict(self.named_parameters())
        table = [n for n, _, _ in rt.params]
        if list(named.keys()) != table:
            raise RuntimeError("parameter table mismatch between module and native graph")
        arena = torch.empty(rt.n_param_floats, dtype=torch.float32, device=dev)
        plist = []
        with torch.no_grad():
            for name, shape, off in rt.params:
                p = named[name]
                if tuple(p.shape) != tuple(shape):
                    raise RuntimeError(f"{name}: shape {tuple(p.shape)} != native {shape}")
                n = p.numel()
                arena[off:off + n].copy_(p.detach().reshape(-1).to(dev, torch.float32))
                p.data = arena[off:off + n].view(shape)
                plist.append((p, off, shape))
            bns = self._bn_modules()
            bn_arena = torch.empty(rt.n_bn_floats, dtype=torch.float32, device=dev)
            nbt = torch.zeros(len(rt.bn), dtype=torch.int64, device=dev)
            for i, (name, ch, off) in enumerate(rt.bn):
                m = bns[name]
                bn_arena[off:off + ch].copy_(m.running_mean.reshape(-1).float())
                bn_arena[off + ch:off + 2 * ch].copy_(m.running_var.reshape(-1).float())
                nbt[i].copy_(m.num_batches_tracked.reshape(()))
                m.running_mean = bn_arena[off:off + ch]
                m.running_var = bn_arena[off + ch:off + 2 * ch]
                m.num_batches_tracked = nbt[i]
        self._state = _ArenaState(rt, plist, arena, bn_arena, nbt)
        return self._state

    def _apply(self, fn, *args, **kwargs):
        self._state = None  # any device / dtype move invalidates the arenas
        return super()._apply(fn, *args, **kwargs)

    # ---------------------------------------------------------------- forward
    def forward(self, x):
        """(N, in_channels, H, W) fp32 -> logits (N, out_channels, H, W) (models/model.py:53-73,
        models/mod.py:53-66).  H and W must be multiples of max(16, 2**depth)."""
        st = self.flatten_()
        if x.dim() != 4 or x.shape[1] != self.in_channels:
            raise ValueError(f"expected (N, {self.in_channels}, H, W), got {tuple(x.shape)}")
        if x.device != st.param_arena.device:
            raise ValueError(f"input on {x.device}, model on {st.param_arena.device}")
        x = x.contiguous().float()
        need_grad = self.training and torch.is_grad_enabled() and any(
            p.requires_grad for p, _, _ in st.params)
        if need_grad:
            return UNetFunction.apply(x, st, *[p for p, _, _ in st.params])
        st.sync_params()
        logits, _ = st.rt.forward(st.param_arena, st.bn_arena, st.nbt_arena, x,
                                  training=self.training)
        return logits

    def params_changed(self):
        """Declare parameter writes the version counters cannot see (through `.data`): the next
        forward repacks the native weight images."""
        st = self._state
        if st is not None:
            st.rt.params_changed()
            st.native_version = None

    @property
    def flat_params(self):
        return self.flatten_().param_arena


class UNet(_HipUNet):
    """models/model.py:5-73."""

    _name = "models.model.UNet"

    def __init__(self, in_channels=1, out_channels=1):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.encoder1 = _conv_block(in_channels, 64)
        self.encoder2 = _conv_block(64, 128)
        self.encoder3 = _conv_block(128, 256)
        self.encoder4 = _conv_block(256, 512)
        self.middle = nn.Sequential(nn.MaxPool2d(kernel_size=2, stride=2), _conv_block(512, 1024),
                                    nn.ConvTranspose2d(1024, 512, kernel_size=2, stride=2))
        self.decoder3 = _upconv_block(1024, 256)
        self.decoder2 = _upconv_block(512, 128)
        self.decoder1 = _upconv_block(256, 64)
        self.final = nn.Sequential(_conv_block(128, 64), nn.Conv2d(64, out_channels, kernel_size=1))
        self._state = None

    def _native_cfg(self):
        return self.in_channels, self.out_channels, _lib.VARIANT_MODEL, 0, 0, _lib.MATH_F32


def _mod_block(cin, cout):
    # models/mod.py:43-51: Conv3x3(no bias) -> BN -> ReLU -> Conv3x3(no bias) -> BN -> ReLU
    return nn.Sequential(nn.Conv2d(cin, cout, kernel_size=3, padding=1, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
                         nn.Conv2d(cout, cout, kernel_size=3, padding=1, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class ModUNet(_HipUNet):
    """models/mod.py:9-66 ``UNet(in_channels, out_channels, base_filters, depth)``.

    Supported here: in_channels 1, out_channels 1..4, base_filters a multiple of 8 up to
    256 (32 / 64 / 128 / 256 natively; the reference grid's 16 / 24 / 48 run zero-padded to
    the next power of two >= 32 inside the library), depth 1..6.

    ``mfma_dtype``: "fp32" (default; exact f32 products like the reference) or "bf16"
    (BASELINE config 4: conv GEMM operands rounded to bf16, f32 accumulate; parameters,
    activations, BN and the optimizer stay f32)."""

    _name = "models.mod.UNet"

    def __init__(self, in_channels=1, out_channels=1, base_filters=64, depth=5,
                 mfma_dtype="fp32", **kwargs):
        super().__init__()
        if str(mfma_dtype) not in ("fp32", "bf16", "torch.float32", "torch.bfloat16"):
            raise ValueError(f"mfma_dtype must be 'fp32' or 'bf16', got {mfma_dtype!r}")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.base_filters, self.depth = base_filters, depth
        self.mfma_dtype = "bf16" if "bf" in str(mfma_dtype) else "fp32"
        # same construction (and RNG consumption) order as mod.py:21-41
        self.encoders = nn.ModuleList()
        self.pools = nn.ModuleList()
        prev = in_channels
        channels = [base_filters * (2 ** i) for i in range(depth)]
        for ch in channels:
            self.encoders.append(_mod_block(prev, ch))
            self.pools.append(nn.MaxPool2d(2, 2))
            prev = ch
        self.bottleneck = _mod_block(prev, prev * 2)
        self.upconvs = nn.ModuleList()
        self.decoders = nn.ModuleList()
        prev = channels[-1] * 2
        for ch in channels[::-1]:
            self.upconvs.append(nn.ConvTranspose2d(prev, ch, kernel_size=2, stride=2))
            self.decoders.append(_mod_block(prev, ch))
            prev = ch
        self.final_conv = nn.Conv2d(base_filters, out_channels, kernel_size=1)
        self._state = None

    def _native_cfg(self):
        return (self.in_channels, self.out_channels, _lib.VARIANT_MOD, self.base_filters,
                self.depth, _lib.MATH_BF16 if self.mfma_dtype == "bf16" else _lib.MATH_F32)


class _ResidualBlock(nn.Module):
    # models/mod.py:71-86 (module tree only; the block runs natively)
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(in_ch, out_ch, 3, padding=1, bias=False), nn.BatchNorm2d(out_ch),
            nn.ReLU(inplace=True),
            nn.Conv2d(out_ch, out_ch, 3, padding=1, bias=False), nn.BatchNorm2d(out_ch))
        self.skip = nn.Conv2d(in_ch, out_ch, 1, bias=False)
        self.relu = nn.ReLU(inplace=True)


class ResUNet(_HipUNet):
    """models/mod.py:88-131 ``ResUNet(in_channels, out_channels, base_filters, depth)``:
    every block is ReLU(conv(x) + skip(x)) with conv = Conv-BN-ReLU-Conv-BN and a bias-free
    1x1 skip.  Same widths as ``ModUNet`` (f32 GEMMs)."""

    _name = "models.mod.ResUNet"

    def __init__(self, in_channels=1, out_channels=1, base_filters=64, depth=5, **kwargs):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.base_filters, self.depth = base_filters, depth
        # construction (and RNG) order of mod.py:96-115
        self.encoders = nn.ModuleList()
        self.pools = nn.ModuleList()
        prev = in_channels
        channels = [base_filters * (2 ** i) for i in range(depth)]
        for ch in channels:
            self.encoders.append(_ResidualBlock(prev, ch))
            self.pools.append(nn.MaxPool2d(2, 2))
            prev = ch
        self.bottleneck = _ResidualBlock(prev, prev * 2)
        self.upconvs = nn.ModuleList()
        self.decoders = nn.ModuleList()
        prev = channels[-1] * 2
        for ch in channels[::-1]:
            self.upconvs.append(nn.ConvTranspose2d(prev, ch, 2, 2))
            self.decoders.append(_ResidualBlock(prev, ch))
            prev = ch
        self.final_conv = nn.Conv2d(base_filters, out_channels, 1)
        self._state = None

    def _native_cfg(self):
        return (self.in_channels, self.out_channels, _lib.VARIANT_RES, self.base_filters,
                self.depth, _lib.MATH_F32)
