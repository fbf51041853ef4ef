"""torch-CPU restatement of the reference UNet training step (test infra only).

Follows, op for op and in the same order:

* ``models/model.py:5-73``   UNet(in=1, out=1): conv_block = Conv3x3(bias) -> ReLU ->
  BN -> Conv3x3 -> ReLU -> BN (``:33-43``); upconv_block = conv_block(Cin, Cin/2) ->
  ConvTranspose2d(k2, s2) (``:45-51``); middle = MaxPool -> conv_block(512,1024) ->
  ConvT(1024,512) (``:16-20``); concat order ``[up, skip]`` (``:64-70``); head 1x1
  conv (``:28-31``).
* ``nn.BatchNorm2d`` train semantics (eps 1e-5, momentum 0.1, biased batch var for
  normalisation, unbiased for running_var, ``num_batches_tracked += 1``).
* ``utils/trainer.py:37,85`` ``nn.BCEWithLogitsLoss()`` (mean),
  ``models/loss.py:7-24`` ``DiceLoss`` (per-sample soft dice, smooth 1) and
  ``models/loss.py:26-46`` ``FocalTverskyLoss`` (batch-global TP/FP/FN).
* ``utils/trainer.py:90`` weighted loss sum; ``:81-93`` zero_grad/backward/step.
* ``utils/trainer.py:41`` ``AdamW(lr)`` with torch defaults betas (0.9, 0.999),
  eps 1e-8, weight_decay 1e-2, restated as torch's ``_single_tensor_adam``.
* ``utils/trainer.py:101,217`` mask readout ``sigmoid(logits) > 0.5``.

Everything runs with ``torch.nn.functional`` on CPU in fp32; because these are the
same ATen kernels in the same order as the module-based reference, the results are
bit-identical to the reference on the same machine (checked in
``tests/test_oracle.py`` against fixtures written by ``tools/gen_golden.py``).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import weights as W

BN_EPS = 1e-5
BN_MOMENTUM = 0.1


def conv_block_names(prefix):
    return [f"{prefix}.0", f"{prefix}.2", f"{prefix}.3", f"{prefix}.5"]


def param_spec(in_channels=1, out_channels=1):
    """(name, shape, kind[, fan_in]) in ``named_parameters()`` order of models/model.py:UNet."""
    spec = []

    def block(prefix, cin, cout):
        spec.append((f"{prefix}.0.weight", (cout, cin, 3, 3), "conv_w"))
        spec.append((f"{prefix}.0.bias", (cout,), "conv_b", cin * 9))
        spec.append((f"{prefix}.2.weight", (cout,), "bn_w"))
        spec.append((f"{prefix}.2.bias", (cout,), "bn_b"))
        spec.append((f"{prefix}.3.weight", (cout, cout, 3, 3), "conv_w"))
        spec.append((f"{prefix}.3.bias", (cout,), "conv_b", cout * 9))
        spec.append((f"{prefix}.5.weight", (cout,), "bn_w"))
        spec.append((f"{prefix}.5.bias", (cout,), "bn_b"))

    def convT(name, cin, cout):
        spec.append((f"{name}.weight", (cin, cout, 2, 2), "convT_w"))
        spec.append((f"{name}.bias", (cout,), "convT_b", cout * 4))

    block("encoder1", in_channels, 64)
    block("encoder2", 64, 128)
    block("encoder3", 128, 256)
    block("encoder4", 256, 512)
    block("middle.1", 512, 1024)
    convT("middle.2", 1024, 512)
    block("decoder3.0", 1024, 512)
    convT("decoder3.1", 512, 256)
    block("decoder2.0", 512, 256)
    convT("decoder2.1", 256, 128)
    block("decoder1.0", 256, 128)
    convT("decoder1.1", 128, 64)
    block("final.0", 128, 64)
    spec.append(("final.1.weight", (out_channels, 64, 1, 1), "conv_w"))
    spec.append(("final.1.bias", (out_channels,), "conv_b", 64))
    return spec


BN_LAYERS = [f"{p}.{i}" for p in ["encoder1", "encoder2", "encoder3", "encoder4", "middle.1",
                                  "decoder3.0", "decoder2.0", "decoder1.0", "final.0"]
             for i in (2, 5)]
BN_CHANNELS = [c for c in [64, 128, 256, 512, 1024, 512, 256, 128, 64] for _ in range(2)]


def init_buffers():
    """Fresh BN buffers (running_mean=0, running_var=1, num_batches_tracked=0)."""
    buf = {}
    for name, c in zip(BN_LAYERS, BN_CHANNELS):
        buf[f"{name}.running_mean"] = torch.zeros(c)
        buf[f"{name}.running_var"] = torch.ones(c)
        buf[f"{name}.num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    return buf


def make_params(seed=42, gamma_lo=0.5, gamma_hi=1.5, in_channels=1, out_channels=1):
    p = W.make_params(param_spec(in_channels, out_channels), seed, gamma_lo, gamma_hi)
    return {k: torch.from_numpy(v) for k, v in p.items()}


def _bn(x, P, B, name, training):
    # nn.BatchNorm2d.forward -> F.batch_norm (torch/nn/modules/batchnorm.py); the module
    # increments num_batches_tracked before the call when training.
    if training:
        B[f"{name}.num_batches_tracked"].add_(1)
    return F.batch_norm(x, B[f"{name}.running_mean"], B[f"{name}.running_var"],
                        P[f"{name}.weight"], P[f"{name}.bias"], training, BN_MOMENTUM, BN_EPS)


_RECORD = None  # test hook: list collecting the post-ReLU (pre-BN) output of every conv
# test hook: 18 boolean masks (NCHW, forward order) replacing the ReLU decisions -- ReLU(z)
# becomes z * mask -- so an fp64 evaluation can follow another evaluation's ReLU branches
# (tests/test_gpu_x3.py: near-zero pre-activations that round to the other side of 0 in f32
# would otherwise move whole upstream gradients)
_RELU_MASKS = None


# test hook: 4 max-pool winner indices (N, C, Ho, Wo, window position 0..3 in torch's scan
# order), so the fp64 evaluation also follows another evaluation's pooling branches (near-ties
# between BN outputs)
_POOL_IDX = None


def _maxpool(x):
    if _POOL_IDX is None:
        return F.max_pool2d(x, 2)
    N, C, H, W = x.shape
    win = x.reshape(N, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, C, H // 2, W // 2, 4)
    return win.gather(-1, _POOL_IDX.pop(0).long().unsqueeze(-1)).squeeze(-1)


def _relu(x):
    if _RELU_MASKS is None:
        return F.relu(x)
    return x * _RELU_MASKS.pop(0).to(x.dtype)


def _conv_block(x, P, B, prefix, training):
    # models/model.py:33-43
    x = F.conv2d(x, P[f"{prefix}.0.weight"], P[f"{prefix}.0.bias"], padding=1)
    x = _relu(x)
    if _RECORD is not None:
        _RECORD.append(x.detach())
    x = _bn(x, P, B, f"{prefix}.2", training)
    x = F.conv2d(x, P[f"{prefix}.3.weight"], P[f"{prefix}.3.bias"], padding=1)
    x = _relu(x)
    if _RECORD is not None:
        _RECORD.append(x.detach())
    x = _bn(x, P, B, f"{prefix}.5", training)
    return x


def _convT(x, P, name):
    return F.conv_transpose2d(x, P[f"{name}.weight"], P[f"{name}.bias"], stride=2)


def forward(x, P, B, training=True, record=None, relu_masks=None, pool_idx=None):
    """models/model.py:53-73.  P: params (name -> tensor), B: buffers (mutated in train mode).
    record: optional list that receives the 18 post-ReLU conv outputs (test diagnostics).
    relu_masks / pool_idx: optional 18 boolean NCHW masks / 4 winner-index tensors that replace
    the conv ReLUs' / max-pools' decisions (test hook)."""
    global _RECORD, _RELU_MASKS, _POOL_IDX
    _RECORD = record
    _RELU_MASKS = None if relu_masks is None else list(relu_masks)
    _POOL_IDX = None if pool_idx is None else list(pool_idx)
    try:
        return _forward(x, P, B, training)
    finally:
        _RECORD = None
        _RELU_MASKS = None
        _POOL_IDX = None


def _forward(x, P, B, training):
    enc1 = _conv_block(x, P, B, "encoder1", training)
    enc2 = _conv_block(_maxpool(enc1), P, B, "encoder2", training)     # F.max_pool2d(enc1, 2)
    enc3 = _conv_block(_maxpool(enc2), P, B, "encoder3", training)
    enc4 = _conv_block(_maxpool(enc3), P, B, "encoder4", training)
    m = _maxpool(enc4)              # middle.0 nn.MaxPool2d(kernel_size=2, stride=2)
    m = _conv_block(m, P, B, "middle.1", training)
    dec4 = _convT(m, P, "middle.2")
    dec4 = torch.cat([dec4, enc4], dim=1)
    dec3 = _convT(_conv_block(dec4, P, B, "decoder3.0", training), P, "decoder3.1")
    dec3 = torch.cat([dec3, enc3], dim=1)
    dec2 = _convT(_conv_block(dec3, P, B, "decoder2.0", training), P, "decoder2.1")
    dec2 = torch.cat([dec2, enc2], dim=1)
    dec1 = _convT(_conv_block(dec2, P, B, "decoder1.0", training), P, "decoder1.1")
    dec1 = torch.cat([dec1, enc1], dim=1)
    f = _conv_block(dec1, P, B, "final.0", training)
    return F.conv2d(f, P["final.1.weight"], P["final.1.bias"])


def bce_with_logits(logits, targets):
    # utils/trainer.py:37 nn.BCEWithLogitsLoss() (reduction='mean')
    return F.binary_cross_entropy_with_logits(logits, targets)


def dice_loss(logits, targets, smooth=1.0):
    # models/loss.py:13-24
    probs = torch.sigmoid(logits)
    probs = probs.view(probs.shape[0], -1)
    targets = targets.view(targets.shape[0], -1).float()
    intersection = (probs * targets).sum(dim=1)
    union = probs.sum(dim=1) + targets.sum(dim=1)
    dice = (2. * intersection + smooth) / (union + smooth)
    return 1 - dice.mean()


def focal_tversky(logits, targets, alpha=0.4, beta=0.6, gamma=2.0, smooth=1e-6):
    # models/loss.py:26-46 FocalTverskyLoss (defaults as utils/trainer.py:38): TP/FP/FN over
    # the WHOLE batch (flattened), ti = (TP+s)/(TP + a FP + b FN + s), loss = (1-ti)^gamma
    probs = torch.sigmoid(logits)
    probs_flat = probs.view(-1)
    targets_flat = targets.view(-1)
    TP = (probs_flat * targets_flat).sum()
    FP = ((probs_flat) * (1 - targets_flat)).sum()
    FN = ((1 - probs_flat) * targets_flat).sum()
    ti = (TP + smooth) / (TP + alpha * FP + beta * FN + smooth)
    return (1 - ti) ** gamma


def mask_readout(logits):
    # utils/trainer.py:101,217
    return (torch.sigmoid(logits) > 0.5).to(torch.uint8)


class AdamWState:
    """torch.optim.AdamW defaults (utils/trainer.py:41): betas (0.9,0.999), eps 1e-8, wd 1e-2."""

    def __init__(self, params, lr=1e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.step_count = 0
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}

    def step(self, params, grads):
        # torch/optim/adam.py _single_tensor_adam, decoupled weight decay branch
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
                denom = (self.v[k].sqrt() / bc2_sqrt).add_(self.eps)
                p.addcdiv_(self.m[k], denom, value=-step_size)


def train_step(P, B, opt, x, t, w_bce=1.0, w_dice=1.0, shards=1, forward_fn=None, w_focal=0.0,
               focal_abg=(0.4, 0.6, 2.0)):
    """utils/trainer.py:81-93 for one batch.  ``shards`` > 1 emulates nn.DataParallel
    (utils/trainer.py:28-30): the batch is split on dim 0 with torch.chunk (DataParallel's
    scatter; B=3 over 2 replicas gives shards of 2 and 1), every shard runs its own
    train-mode BN, logits are gathered and the loss is taken on the full batch.
    (Only shard 0's running stats are kept, as DP keeps replica 0's.)
    Loss = w_bce*BCE + w_dice*Dice + w_focal*FocalTversky (utils/trainer.py:90; the CLI
    defaults main.py:43-46 are 1/0/1/0).  ``forward_fn`` replaces models/model.py's graph
    (e.g. mod_ref_cpu.make_forward).  Returns dict(logits, loss, bce, dice, focal, grads)."""
    fwd = forward if forward_fn is None else forward_fn
    Pg = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    if shards == 1:
        logits = fwd(x, Pg, B, True)
    else:
        outs = []
        for s, xs in enumerate(torch.chunk(x, shards, dim=0)):
            Bs = B if s == 0 else {k: v.clone() for k, v in B.items()}
            outs.append(fwd(xs, Pg, Bs, True))
        logits = torch.cat(outs, 0)
    bce = bce_with_logits(logits, t)
    dice = dice_loss(logits, t)
    focal = focal_tversky(logits, t, *focal_abg)
    loss = w_bce * bce + w_dice * dice
    if w_focal != 0:
        loss = loss + w_focal * focal
    loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in Pg.items()}
    if opt is not None:
        opt.step(P, grads)
    return dict(logits=logits.detach(), loss=loss.detach(), bce=bce.detach(),
                dice=dice.detach(), focal=focal.detach(), grads=grads)


# ---- analytic FLOP count -------------------------------------------------
def conv_macs_per_image(H, W, in_channels=1, out_channels=1):
    """MACs of all conv / convT layers for one HxW image (forward)."""
    macs = 0
    lv = [(in_channels, 64, 1), (64, 128, 2), (128, 256, 4), (256, 512, 8), (512, 1024, 16)]
    for cin, cout, s in lv:
        hw = (H // s) * (W // s)
        macs += hw * 9 * (cin * cout + cout * cout)
    dec = [(1024, 512, 8), (512, 256, 4), (256, 128, 2), (128, 64, 1)]
    for cin, cout, s in dec:
        hw = (H // s) * (W // s)
        macs += hw * 9 * (cin * cout + cout * cout)
    for cin, cout, s in [(1024, 512, 16), (512, 256, 8), (256, 128, 4), (128, 64, 2)]:
        hw = (H // s) * (W // s)
        macs += hw * cin * cout * 4
    macs += H * W * 64 * out_channels
    return macs


def train_flops_per_image(H, W):
    """fwd + dgrad + wgrad = 3x forward MACs x2, minus encoder1.0's unneeded dgrad."""
    macs = conv_macs_per_image(H, W)
    return 6 * macs - 2 * (H * W * 9 * 64)
