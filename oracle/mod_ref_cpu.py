"""torch-CPU restatement of ``models/mod.py:UNet`` (test infra only).

The variant ``main.py``-style configs reach through ``models/mod.py:9-66`` (SURVEY.md §8
row a19, BASELINE config 4).  Differences from ``models/model.py:UNet`` that the
restatement follows:

* ``_block`` (``mod.py:43-51``): Conv3x3 **without bias** -> BN -> ReLU -> Conv3x3 (no
  bias) -> BN -> ReLU (BN before ReLU).
* ``depth`` encoders of ``base_filters * 2**i`` channels, each followed by MaxPool2d(2)
  (``mod.py:25-30``); bottleneck ``_block(C, 2C)`` (``:32``).
* decoder step (``:59-65``): ConvTranspose2d(k2, s2, bias) **first**, then the concat
  ``[skip, up]`` (skip first), then ``_block(2C, C)``; ``F.interpolate`` only when the
  shapes differ (never for H, W divisible by 2**depth, which the path requires).
* head: ``final_conv`` Conv2d(base, out, 1) with bias (``:41``).

Parameters are named and ordered exactly like ``named_parameters()`` of the reference
module (encoders.*, bottleneck.*, upconvs.*, decoders.*, final_conv.*).  Losses, the
train step and AdamW are shared with ``unet_ref_cpu``.

``make_forward(depth, bf16=True)`` is the checker of the bf16-MFMA build of BASELINE
config 4: every 3x3 conv except the first (Cin = 1) and every ConvTranspose takes its
activation and weight rounded to bf16 (round to nearest even) and, in backward, its output
gradient rounded to bf16 before both the input- and the weight-gradient products; all
sums, BN, ReLU, pooling, the head and the losses stay in the evaluation dtype.  That is
the arithmetic of the HIP bf16 GEMMs (operands rounded when staged into LDS, f32
accumulate), so the two agree to fp32 accumulation-order noise.
"""
import torch
import torch.nn.functional as F

from . import unet_ref_cpu as O
from . import weights as W


def _block_spec(spec, prefix, cin, cout):
    spec.append((f"{prefix}.0.weight", (cout, cin, 3, 3), "conv_w"))
    spec.append((f"{prefix}.1.weight", (cout,), "bn_w"))
    spec.append((f"{prefix}.1.bias", (cout,), "bn_b"))
    spec.append((f"{prefix}.3.weight", (cout, cout, 3, 3), "conv_w"))
    spec.append((f"{prefix}.4.weight", (cout,), "bn_w"))
    spec.append((f"{prefix}.4.bias", (cout,), "bn_b"))


def param_spec(in_channels=1, out_channels=1, base=64, depth=5):
    """(name, shape, kind[, fan_in]) in named_parameters() order of mod.py:UNet."""
    spec = []
    ch = [base * (2 ** i) for i in range(depth)]
    prev = in_channels
    for i, c in enumerate(ch):                       # mod.py:27-30
        _block_spec(spec, f"encoders.{i}", prev, c)
        prev = c
    _block_spec(spec, "bottleneck", prev, 2 * prev)  # mod.py:32
    prev = ch[-1] * 2
    ups = []
    for j, c in enumerate(ch[::-1]):                 # mod.py:37-40
        ups.append((j, prev, c))
        prev = c
    for j, cin, cout in ups:                         # ModuleList `upconvs` registers first
        spec.append((f"upconvs.{j}.weight", (cin, cout, 2, 2), "convT_w"))
        spec.append((f"upconvs.{j}.bias", (cout,), "convT_b", cout * 4))
    for j, cin, cout in ups:
        _block_spec(spec, f"decoders.{j}", cin, cout)
    spec.append(("final_conv.weight", (out_channels, base, 1, 1), "conv_w"))
    spec.append(("final_conv.bias", (out_channels,), "conv_b", base))
    return spec


def bn_layers(base=64, depth=5):
    """[(name, channels)] in named_buffers() order."""
    ch = [base * (2 ** i) for i in range(depth)]
    out = []
    for i, c in enumerate(ch):
        out += [(f"encoders.{i}.1", c), (f"encoders.{i}.4", c)]
    out += [("bottleneck.1", 2 * ch[-1]), ("bottleneck.4", 2 * ch[-1])]
    for j, c in enumerate(ch[::-1]):
        out += [(f"decoders.{j}.1", c), (f"decoders.{j}.4", c)]
    return out


def init_buffers(base=64, depth=5):
    buf = {}
    for name, c in bn_layers(base, depth):
        buf[f"{name}.running_mean"] = torch.zeros(c)
        buf[f"{name}.running_var"] = torch.ones(c)
        buf[f"{name}.num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    return buf


def make_params(seed=42, base=64, depth=5, gamma_lo=0.5, gamma_hi=1.5, in_channels=1,
                out_channels=1):
    p = W.make_params(param_spec(in_channels, out_channels, base, depth), seed, gamma_lo, gamma_hi)
    return {k: torch.from_numpy(v) for k, v in p.items()}


def _rnd(t):
    """Round to bf16 (nearest even) and back to t's dtype."""
    return t.to(torch.bfloat16).to(t.dtype)


class _BF16Operands(torch.autograd.Function):
    """fn(rnd(x), rnd(w)) with backward products on rnd(grad) (see module docstring)."""

    @staticmethod
    def forward(ctx, fn, x, w):
        xr, wr = _rnd(x), _rnd(w)
        ctx.fn = fn
        ctx.save_for_backward(xr, wr)
        return fn(xr, wr)

    @staticmethod
    def backward(ctx, g):
        xr, wr = ctx.saved_tensors
        with torch.enable_grad():
            a = xr.detach().requires_grad_(True)
            b = wr.detach().requires_grad_(True)
            dx, dw = torch.autograd.grad(ctx.fn(a, b), (a, b), _rnd(g))
        return None, dx, dw


def _conv3(x, w, bf16):
    if not bf16:
        return F.conv2d(x, w, None, padding=1)
    return _BF16Operands.apply(lambda a, b: F.conv2d(a, b, None, padding=1), x, w)


def _convT(x, w, b, bf16):
    if not bf16:
        return F.conv_transpose2d(x, w, b, stride=2)
    return _BF16Operands.apply(lambda a, ww: F.conv_transpose2d(a, ww, None, stride=2), x, w) + \
        b.view(1, -1, 1, 1)


def _block(x, P, B, prefix, training, bf16=False, first=False):
    # mod.py:43-51 (the Cin = 1 first conv runs in f32 on the HIP path too)
    x = _conv3(x, P[f"{prefix}.0.weight"], bf16 and not first)
    x = F.relu(O._bn(x, P, B, f"{prefix}.1", training))
    x = _conv3(x, P[f"{prefix}.3.weight"], bf16)
    return F.relu(O._bn(x, P, B, f"{prefix}.4", training))


def make_forward(depth, bf16=False):
    """forward(x, P, B, training) of mod.py:UNet with `depth` levels (mod.py:53-66)."""

    def forward(x, P, B, training=True):
        skips = []
        for i in range(depth):
            x = _block(x, P, B, f"encoders.{i}", training, bf16, first=(i == 0))
            skips.append(x)
            x = F.max_pool2d(x, 2, 2)
        x = _block(x, P, B, "bottleneck", training, bf16)
        for j, skip in enumerate(reversed(skips)):
            x = _convT(x, P[f"upconvs.{j}.weight"], P[f"upconvs.{j}.bias"], bf16)
            if x.shape != skip.shape:
                x = F.interpolate(x, size=skip.shape[2:], mode="bilinear", align_corners=False)
            x = torch.cat([skip, x], dim=1)
            x = _block(x, P, B, f"decoders.{j}", training, bf16)
        return F.conv2d(x, P["final_conv.weight"], P["final_conv.bias"])

    return forward


def train_step(P, B, opt, x, t, depth, w_bce=1.0, w_dice=1.0, shards=1, bf16=False):
    """utils/trainer.py:81-93 with mod.py:UNet as the model."""
    return O.train_step(P, B, opt, x, t, w_bce, w_dice, shards,
                        forward_fn=make_forward(depth, bf16))


# ---------------------------------------------------------------- ResUNet (mod.py:71-131)
def _res_block_spec(spec, prefix, cin, cout):
    # ResidualBlock registers `conv` (Sequential) then `skip` (mod.py:73-83)
    spec.append((f"{prefix}.conv.0.weight", (cout, cin, 3, 3), "conv_w"))
    spec.append((f"{prefix}.conv.1.weight", (cout,), "bn_w"))
    spec.append((f"{prefix}.conv.1.bias", (cout,), "bn_b"))
    spec.append((f"{prefix}.conv.3.weight", (cout, cout, 3, 3), "conv_w"))
    spec.append((f"{prefix}.conv.4.weight", (cout,), "bn_w"))
    spec.append((f"{prefix}.conv.4.bias", (cout,), "bn_b"))
    spec.append((f"{prefix}.skip.weight", (cout, cin, 1, 1), "conv_w"))


def res_param_spec(in_channels=1, out_channels=1, base=64, depth=5):
    """named_parameters() order of mod.py:ResUNet (same layout as UNet, residual blocks)."""
    spec = []
    ch = [base * (2 ** i) for i in range(depth)]
    prev = in_channels
    for i, c in enumerate(ch):
        _res_block_spec(spec, f"encoders.{i}", prev, c)
        prev = c
    _res_block_spec(spec, "bottleneck", prev, 2 * prev)
    prev = ch[-1] * 2
    ups = []
    for j, c in enumerate(ch[::-1]):
        ups.append((j, prev, c))
        prev = c
    for j, cin, cout in ups:
        spec.append((f"upconvs.{j}.weight", (cin, cout, 2, 2), "convT_w"))
        spec.append((f"upconvs.{j}.bias", (cout,), "convT_b", cout * 4))
    for j, cin, cout in ups:
        _res_block_spec(spec, f"decoders.{j}", cin, cout)
    spec.append(("final_conv.weight", (out_channels, base, 1, 1), "conv_w"))
    spec.append(("final_conv.bias", (out_channels,), "conv_b", base))
    return spec


def res_bn_layers(base=64, depth=5):
    """[(name, channels)] in named_buffers() order of mod.py:ResUNet."""
    return [(n[:-2] + ".conv" + n[-2:], c) for n, c in bn_layers(base, depth)]


def res_init_buffers(base=64, depth=5):
    buf = {}
    for name, c in res_bn_layers(base, depth):
        buf[f"{name}.running_mean"] = torch.zeros(c)
        buf[f"{name}.running_var"] = torch.ones(c)
        buf[f"{name}.num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    return buf


def res_make_params(seed=42, base=64, depth=5, gamma_lo=0.5, gamma_hi=1.5, in_channels=1,
                    out_channels=1):
    p = W.make_params(res_param_spec(in_channels, out_channels, base, depth), seed, gamma_lo,
                      gamma_hi)
    return {k: torch.from_numpy(v) for k, v in p.items()}


def _res_block(x, P, B, prefix, training):
    # mod.py:85-86: relu(conv(x) + skip(x)), conv = Conv-BN-ReLU-Conv-BN (mod.py:75-81)
    y = F.conv2d(x, P[f"{prefix}.conv.0.weight"], None, padding=1)
    y = F.relu(O._bn(y, P, B, f"{prefix}.conv.1", training))
    y = F.conv2d(y, P[f"{prefix}.conv.3.weight"], None, padding=1)
    y = O._bn(y, P, B, f"{prefix}.conv.4", training)
    return F.relu(y + F.conv2d(x, P[f"{prefix}.skip.weight"]))


def make_res_forward(depth):
    """forward(x, P, B, training) of mod.py:ResUNet (mod.py:112-124)."""

    def forward(x, P, B, training=True):
        skips = []
        for i in range(depth):
            x = _res_block(x, P, B, f"encoders.{i}", training)
            skips.append(x)
            x = F.max_pool2d(x, 2, 2)
        x = _res_block(x, P, B, "bottleneck", training)
        for j, skip in enumerate(reversed(skips)):
            x = F.conv_transpose2d(x, P[f"upconvs.{j}.weight"], P[f"upconvs.{j}.bias"], stride=2)
            if x.shape != skip.shape:
                x = F.interpolate(x, size=skip.shape[2:], mode="bilinear", align_corners=False)
            x = torch.cat([skip, x], dim=1)
            x = _res_block(x, P, B, f"decoders.{j}", training)
        return F.conv2d(x, P["final_conv.weight"], P["final_conv.bias"])

    return forward


def res_train_step(P, B, opt, x, t, depth, w_bce=1.0, w_dice=1.0, shards=1):
    """utils/trainer.py:81-93 with mod.py:ResUNet (the model main.py:122 builds)."""
    return O.train_step(P, B, opt, x, t, w_bce, w_dice, shards, forward_fn=make_res_forward(depth))


def conv_macs_per_image(H, W, in_channels=1, out_channels=1, base=64, depth=5):
    macs = 0
    prev = in_channels
    for i in range(depth + 1):                    # encoders + bottleneck
        c = base << i
        hw = (H >> i) * (W >> i)
        macs += hw * 9 * (prev * c + c * c)
        prev = c
    for l in range(depth - 1, -1, -1):            # upconv into level l, then the block
        c = base << l
        hw_in = (H >> (l + 1)) * (W >> (l + 1))
        macs += hw_in * (2 * c) * c * 4
        hw = (H >> l) * (W >> l)
        macs += hw * 9 * (2 * c * c + c * c)
    macs += H * W * base * out_channels
    return macs


def train_flops_per_image(H, W, base=64, depth=5):
    """fwd + dgrad + wgrad minus the first conv's unneeded dgrad."""
    return 6 * conv_macs_per_image(H, W, base=base, depth=depth) - 2 * (H * W * 9 * base)
