#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REAL reference.

Runs only in the build container (it imports /root/reference, which never travels
to the GPU box).  The reference modules used are imported unmodified:

* ``models/model.py``  UNet                     (the network)
* ``models/loss.py``   DiceLoss                 (Dice term)
* ``torch.nn.BCEWithLogitsLoss``                (utils/trainer.py:37)
* ``torch.optim.AdamW(params, lr)``             (utils/trainer.py:41)

The step body mirrors ``utils/trainer.py:81-93`` (zero_grad, forward, losses,
weighted sum with bce_ratio=dice_ratio=1, backward, optimizer.step).  Weights and
inputs come from ``oracle/weights.py`` (counter hash), so the fixtures can be
re-derived anywhere without the reference; only the *outputs* need it.

Fixtures (all float64 statistics computed from fp32 results):
  unet_b2_64.npz    B=2, 1x64x64, 3 AdamW steps: full logits, masks, losses, per-tensor
                    grad norm/sum/samples, param samples after every step, running stats,
                    eval-mode logits after step 3.
  unet_b2_256.npz   B=2, 1x256x256, one step: logit samples/stats, packed mask, losses,
                    grad norm/sum/samples.
  unet_dp2_64.npz   B=4, 1x64x64 split into 2 DataParallel-style shards (per-shard BN,
                    full-batch loss): losses and grad norm/sum/samples.
  unet_neg_32.npz   B=2, 1x32x32 with BN gamma in [-1, 1] (max-pool after a sign flip),
                    one step: full logits, grad norm/sum/samples.
  mod_d3_64.npz     models/mod.py UNet(base 64, depth 3), B=2 1x64x64, 2 AdamW steps
                    (lr 1e-4): full logits, masks, losses, grad norm/sum/samples, param
                    samples, running stats; gamma in [-1, 1] on a second case (neg_*).
  res_d3_64.npz     models/mod.py ResUNet(base 64, depth 3) (what main.py:122 builds, at
                    reduced depth), B=2 1x64x64, 2 AdamW steps (lr 1e-4): as mod_d3_64.
  mod_c4_64.npz     models/mod.py UNet(base 128, depth 5) -- the config-4 architecture,
                    497,438,849 params -- at B=2 1x64x64, one step: full logits, losses,
                    grad norm/sum/samples.
  unet_focal_64.npz the reference CLI's default loss mix (main.py:43-46: bce 1, dice 0,
                    focal 1, boundary 0) with the real FocalTverskyLoss() (trainer.py:38),
                    B=2 1x64x64, 3 AdamW steps (utils/trainer.py:81-93): full logits, the
                    three loss terms, grad norm/sum/samples, param samples.
  mod_narrow_64.npz the reference grid's narrow widths (config/config.yaml): models/mod.py
                    UNet(base 32, depth 4) two AdamW steps (lr 1e-4) with full logits,
                    losses, grad norm/sum/samples, param samples, running stats, eval
                    logits (prefix b32_); one step of UNet(base 24, depth 3) (u24_),
                    UNet(base 48, depth 3) (u48_) and ResUNet(base 16, depth 3) (r16_).
  unet_dpf_64.npz   nn.DataParallel with FocalTversky in the loss (the loss of the gathered
                    logits, global TP/FP/FN): eq_* B=4 in 2 shards of 2, ratios 1/0/1/0;
                    uneq_* B=3 in shards of 2 and 1 (DataParallel's chunked scatter), ratios
                    1/1/1/0.  Losses and grad norm/sum/samples.
  unet_dpe_64.npz   nn.DataParallel training THEN evaluation (utils/trainer.py:28-30, 47-119,
                    121-172, 206-250): Trainer.train_one_epoch over SyntheticSegmentation(5, 64,
                    seed=4) at global batch 4 (shards 2+2, then 1 sample on replica 0 only),
                    the CLI default loss mix 1/0/1/0 (starting from running statistics warmed by 30
                    train-mode passes, stored as init_*), then validate (seed 5) and test (seed 6)
                    in eval mode, where DataParallel re-replicates module 0 so every shard
                    uses replica 0's running statistics.  lr0_: lr = 0 (parameters fixed, only
                    the BN buffers move: a strict pin of the buffer semantics); lr4_: lr =
                    1e-4.  Running stats, val / test logits, per-batch val losses, counts.
  modres_dp_64.npz  nn.DataParallel training of the networks the reference CLI builds:
                    ResUNet(64, 3) (res_, main.py:122) and mod.py UNet(64, 3) (mod_), B = 3
                    over two replicas (shards 2 + 1), BCE + Dice of the gathered logits, two
                    AdamW steps (lr 1e-4): logits, losses, grad norm/sum/samples, param
                    samples, running stats per step; eval logits with replica 0's buffers.
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

from models.model import UNet as RefUNet  # noqa: E402  (reference)
from models.loss import DiceLoss as RefDice  # noqa: E402  (reference)
from models.loss import FocalTverskyLoss as RefFocal  # noqa: E402  (reference, models/loss.py:26-46)
from models.mod import UNet as RefModUNet  # noqa: E402  (reference, models/mod.py:9-66)
from models.mod import ResUNet as RefResUNet  # noqa: E402  (reference, models/mod.py:88-131)

from oracle import weights as W  # noqa: E402
from oracle import unet_ref_cpu as O  # noqa: E402
from oracle import mod_ref_cpu as MO  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
NSAMP = 64


def sample_idx(t, n):
    return np.floor(W.uniform(7, 3000 + t, NSAMP) * n).astype(np.int64)


def build(seed=42, gamma_lo=0.5, gamma_hi=1.5):
    torch.manual_seed(0)
    m = RefUNet(1, 1)
    params = O.make_params(seed, gamma_lo, gamma_hi)
    names = [n for n, _ in m.named_parameters()]
    assert names == [s[0] for s in O.param_spec()], "param order mismatch"
    sd = m.state_dict()
    for k, v in params.items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    return m


def grad_stats(m, prefix, out):
    names, norms, sums, samp = [], [], [], []
    for t, (n, p) in enumerate(m.named_parameters()):
        g = p.grad.detach().double().reshape(-1)
        names.append(n)
        norms.append(g.norm().item())
        sums.append(g.sum().item())
        samp.append(g[torch.from_numpy(sample_idx(t, g.numel()))].numpy())
    out[f"{prefix}grad_norm"] = np.array(norms)
    out[f"{prefix}grad_sum"] = np.array(sums)
    out[f"{prefix}grad_samp"] = np.stack(samp)


def param_samples(m):
    return np.stack([p.detach().reshape(-1)[torch.from_numpy(sample_idx(t, p.numel()))].numpy()
                     for t, (_, p) in enumerate(m.named_parameters())])


def step(m, opt, x, t, dice):
    bce = torch.nn.BCEWithLogitsLoss()
    opt.zero_grad()
    logits = m(x)
    lb = bce(logits, t)
    ld = dice(logits, t)
    loss = 1.0 * lb + 1.0 * ld
    loss.backward()
    opt.step()
    return logits.detach(), lb.item(), ld.item(), loss.item()


def case_b2_64():
    m = build()
    m.train()
    x = torch.from_numpy(W.make_input(1, 2, 1, 64, 64))
    t = torch.from_numpy(W.make_target(1, 2, 64, 64))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-5)
    dice = RefDice()
    out = dict(x=x.numpy(), t=t.numpy(), param_names=np.array([n for n, _ in m.named_parameters()]))
    out["params0_samp"] = param_samples(m)
    for s in range(3):
        logits, lb, ld, loss = step(m, opt, x, t, dice)
        out[f"s{s}_logits"] = logits.numpy()
        out[f"s{s}_mask"] = (torch.sigmoid(logits) > 0.5).numpy().astype(np.uint8)
        out[f"s{s}_bce"], out[f"s{s}_dice"], out[f"s{s}_loss"] = lb, ld, loss
        grad_stats(m, f"s{s}_", out)
        out[f"s{s}_params_samp"] = param_samples(m)
        bufs = dict(m.named_buffers())
        out[f"s{s}_running_mean"] = np.concatenate([bufs[f"{n}.running_mean"].numpy() for n in O.BN_LAYERS])
        out[f"s{s}_running_var"] = np.concatenate([bufs[f"{n}.running_var"].numpy() for n in O.BN_LAYERS])
        out[f"s{s}_nbt"] = np.array([bufs[f"{n}.num_batches_tracked"].item() for n in O.BN_LAYERS])
    m.eval()
    with torch.no_grad():
        out["eval_logits"] = m(x).numpy()
    np.savez_compressed(os.path.join(OUT, "unet_b2_64.npz"), **out)


def case_b2_256():
    m = build()
    m.train()
    x = torch.from_numpy(W.make_input(2, 2, 1, 256, 256))
    t = torch.from_numpy(W.make_target(2, 2, 256, 256))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-5)
    logits, lb, ld, loss = step(m, opt, x, t, RefDice())
    flat = logits.reshape(-1)
    li = np.floor(W.uniform(9, 4000, 4096) * flat.numel()).astype(np.int64)
    out = dict(logit_idx=li, logit_samp=flat[torch.from_numpy(li)].numpy(),
               logit_max_abs=flat.abs().max().item(), logit_sum=flat.double().sum().item(),
               logit_norm=flat.double().norm().item(),
               mask_bits=np.packbits((torch.sigmoid(logits) > 0.5).numpy().astype(np.uint8).reshape(-1)),
               bce=lb, dice=ld, loss=loss)
    grad_stats(m, "", out)
    np.savez_compressed(os.path.join(OUT, "unet_b2_256.npz"), **out)


def case_dp2_64():
    """nn.DataParallel numerics (utils/trainer.py:28-30): scatter dim 0, per-replica BN,
    gather logits, loss on the full batch, grads summed over replicas."""
    m = build()
    m.train()
    x = torch.from_numpy(W.make_input(3, 4, 1, 64, 64))
    t = torch.from_numpy(W.make_target(3, 4, 64, 64))
    bns = [mod for mod in m.modules() if isinstance(mod, torch.nn.BatchNorm2d)]
    bufs0 = [(b.running_mean.clone(), b.running_var.clone(), b.num_batches_tracked.clone()) for b in bns]
    outs = []
    for s, xs in enumerate(torch.chunk(x, 2, 0)):
        if s > 0:  # replica s>0 gets its own broadcast copy of the buffers; replica 0's are kept
            keep = [(b.running_mean, b.running_var, b.num_batches_tracked) for b in bns]
            for b, (rm, rv, nb) in zip(bns, bufs0):
                b.running_mean, b.running_var, b.num_batches_tracked = rm.clone(), rv.clone(), nb.clone()
        outs.append(m(xs))
        if s > 0:
            for b, (rm, rv, nb) in zip(bns, keep):
                b.running_mean, b.running_var, b.num_batches_tracked = rm, rv, nb
    logits = torch.cat(outs, 0)
    lb = torch.nn.BCEWithLogitsLoss()(logits, t)
    ld = RefDice()(logits, t)
    loss = lb + ld
    loss.backward()
    out = dict(bce=lb.item(), dice=ld.item(), loss=loss.item(), logits=logits.detach().numpy())
    grad_stats(m, "", out)
    np.savez_compressed(os.path.join(OUT, "unet_dp2_64.npz"), **out)


def step_ratios(m, opt, x, t, w_bce, w_dice, w_focal):
    """utils/trainer.py:81-93 with the reference's loss objects and weights (:85-90)."""
    bce, dice, focal = torch.nn.BCEWithLogitsLoss(), RefDice(), RefFocal()
    if opt is not None:
        opt.zero_grad()
    logits = m(x)
    lb, ld, lf = bce(logits, t), dice(logits, t), focal(logits, t)
    loss = w_bce * lb + w_dice * ld + w_focal * lf
    loss.backward()
    if opt is not None:
        opt.step()
    return logits.detach(), lb.item(), ld.item(), lf.item(), loss.item()


def case_focal_64():
    m = build()
    m.train()
    x = torch.from_numpy(W.make_input(21, 2, 1, 64, 64))
    t = torch.from_numpy(W.make_target(21, 2, 64, 64))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-5)
    out = dict(x=x.numpy(), t=t.numpy())
    for s in range(3):
        logits, lb, ld, lf, loss = step_ratios(m, opt, x, t, 1.0, 0.0, 1.0)
        p = f"s{s}_"
        out[p + "logits"] = logits.numpy()
        out[p + "bce"], out[p + "dice"], out[p + "focal"], out[p + "loss"] = lb, ld, lf, loss
        grad_stats(m, p, out)
        out[p + "params_samp"] = param_samples(m)
    np.savez_compressed(os.path.join(OUT, "unet_focal_64.npz"), **out)


def dp_forward(m, x, shards):
    """nn.DataParallel forward (utils/trainer.py:28-30): torch.chunk scatter, per-replica BN
    (replica 0 keeps its running stats), logits gathered on dim 0."""
    bns = [mod for mod in m.modules() if isinstance(mod, torch.nn.BatchNorm2d)]
    bufs0 = [(b.running_mean.clone(), b.running_var.clone(), b.num_batches_tracked.clone()) for b in bns]
    outs = []
    for s, xs in enumerate(torch.chunk(x, shards, 0)):
        if s > 0:
            keep = [(b.running_mean, b.running_var, b.num_batches_tracked) for b in bns]
            for b, (rm, rv, nb) in zip(bns, bufs0):
                b.running_mean, b.running_var, b.num_batches_tracked = rm.clone(), rv.clone(), nb.clone()
        outs.append(m(xs))
        if s > 0:
            for b, (rm, rv, nb) in zip(bns, keep):
                b.running_mean, b.running_var, b.num_batches_tracked = rm, rv, nb
    return torch.cat(outs, 0)


def case_dp_focal_64():
    out = {}
    for tag, B, ratios, seed in (("eq_", 4, (1.0, 0.0, 1.0), 22), ("uneq_", 3, (1.0, 1.0, 1.0), 23)):
        m = build()
        m.train()
        x = torch.from_numpy(W.make_input(seed, B, 1, 64, 64))
        t = torch.from_numpy(W.make_target(seed, B, 64, 64))
        logits = dp_forward(m, x, 2)
        lb = torch.nn.BCEWithLogitsLoss()(logits, t)
        ld = RefDice()(logits, t)
        lf = RefFocal()(logits, t)
        loss = ratios[0] * lb + ratios[1] * ld + ratios[2] * lf
        loss.backward()
        out[tag + "ratios"] = np.array(ratios)
        out[tag + "bce"], out[tag + "dice"], out[tag + "focal"], out[tag + "loss"] = (
            lb.item(), ld.item(), lf.item(), loss.item())
        out[tag + "logits"] = logits.detach().numpy()
        grad_stats(m, tag, out)
    np.savez_compressed(os.path.join(OUT, "unet_dpf_64.npz"), **out)


def _synthetic(n, seed):
    sys.path.insert(0, os.path.join(REPO, "thyroid-nodule-image-segmentation-unet-ddti_amd"))
    from data.data_loader import SyntheticSegmentation
    ds = SyntheticSegmentation(n, 64, seed=seed)
    return (torch.stack([ds[i][0] for i in range(n)]), torch.stack([ds[i][1] for i in range(n)]))


def case_dp_eval_64():
    out = {}
    xtr, ttr = _synthetic(5, 4)
    xva, tva = _synthetic(5, 5)
    xte, tte = _synthetic(5, 6)
    bce, dice, focal = torch.nn.BCEWithLogitsLoss(), RefDice(), RefFocal()
    for tag, lr in (("lr0_", 0.0), ("lr4_", 1e-4)):
        m = build()
        m.train()
        with torch.no_grad():  # warm the running statistics (fresh ones give constant eval
            for _ in range(30):  # logits); the test loads these as the starting buffers
                m(xtr)
        bufs = dict(m.named_buffers())
        out[tag + "init_running_mean"] = np.concatenate([bufs[f"{n}.running_mean"].numpy() for n in O.BN_LAYERS])
        out[tag + "init_running_var"] = np.concatenate([bufs[f"{n}.running_var"].numpy() for n in O.BN_LAYERS])
        out[tag + "init_nbt"] = np.array([bufs[f"{n}.num_batches_tracked"].item() for n in O.BN_LAYERS])
        opt = torch.optim.AdamW(m.parameters(), lr=lr)
        for sl in (slice(0, 4), slice(4, 5)):  # Trainer.train_one_epoch, DataParallel step
            opt.zero_grad()
            logits = dp_forward(m, xtr[sl], 2)
            loss = 1.0 * bce(logits, ttr[sl]) + 0.0 * dice(logits, ttr[sl]) + 1.0 * focal(logits, ttr[sl])
            loss.backward()
            opt.step()
        bufs = dict(m.named_buffers())
        out[tag + "running_mean"] = np.concatenate([bufs[f"{n}.running_mean"].numpy() for n in O.BN_LAYERS])
        out[tag + "running_var"] = np.concatenate([bufs[f"{n}.running_var"].numpy() for n in O.BN_LAYERS])
        out[tag + "params_samp"] = param_samples(m)
        m.eval()
        with torch.no_grad():
            vl = m(xva)  # == the gathered per-shard eval forwards (eval BN is per sample)
            tl = m(xte)
            vloss = []
            for sl in (slice(0, 4), slice(4, 5)):  # Trainer.validate's per-batch losses
                lb, ld, lf = bce(vl[sl], tva[sl]), dice(vl[sl], tva[sl]), focal(vl[sl], tva[sl])
                vloss.append([lb.item(), ld.item(), lf.item(), (lb + 0.0 * ld + lf).item(), sl.stop - sl.start])
        out[tag + "val_logits"] = vl.numpy()
        out[tag + "val_losses"] = np.array(vloss)
        out[tag + "test_logits"] = tl.numpy()
        for k, lg, tg in (("val_", vl, tva), ("test_", tl, tte)):
            pr = (torch.sigmoid(lg) > 0.5).numpy().reshape(-1)
            # validate: targets cast to int (utils/utils.py:240-251); test: astype(uint8)
            # (utils/trainer.py:220,236-242); both {0, 1} here
            tgi = tg.numpy().astype(np.uint8).reshape(-1)
            out[tag + k + "counts"] = np.array([(pr & (tgi == 1)).sum(), (pr & (tgi == 0)).sum(),
                                                (~pr & (tgi == 1)).sum(), (~pr & (tgi == 0)).sum()])
    np.savez_compressed(os.path.join(OUT, "unet_dpe_64.npz"), **out)


def case_neg_32():
    m = build(seed=5, gamma_lo=-1.0, gamma_hi=1.0)
    m.train()
    x = torch.from_numpy(W.make_input(4, 2, 1, 32, 32))
    t = torch.from_numpy(W.make_target(4, 2, 32, 32))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-5)
    logits, lb, ld, loss = step(m, opt, x, t, RefDice())
    out = dict(logits=logits.numpy(), bce=lb, dice=ld, loss=loss)
    grad_stats(m, "", out)
    np.savez_compressed(os.path.join(OUT, "unet_neg_32.npz"), **out)


def build_mod(base, depth, seed=42, gamma_lo=0.5, gamma_hi=1.5):
    torch.manual_seed(0)
    m = RefModUNet(1, 1, base_filters=base, depth=depth)
    spec = MO.param_spec(1, 1, base, depth)
    assert [n for n, _ in m.named_parameters()] == [s[0] for s in spec], "mod param order"
    assert [n for n, _ in m.named_buffers() if n.endswith("running_mean")] == \
        [f"{n}.running_mean" for n, _ in MO.bn_layers(base, depth)], "mod buffer order"
    params = MO.make_params(seed, base, depth, gamma_lo, gamma_hi)
    sd = m.state_dict()
    for k, v in params.items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    return m


def case_mod_d3_64():
    out = {}
    for tag, (seed, lo, hi) in (("", (42, 0.5, 1.5)), ("neg_", (5, -1.0, 1.0))):
        m = build_mod(64, 3, seed, lo, hi)
        m.train()
        x = torch.from_numpy(W.make_input(11, 2, 1, 64, 64))
        t = torch.from_numpy(W.make_target(11, 2, 64, 64))
        opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
        names = [n for n, _ in MO.bn_layers(64, 3)]
        for s in range(2):
            logits, lb, ld, loss = step(m, opt, x, t, RefDice())
            p = f"{tag}s{s}_"
            out[p + "logits"] = logits.numpy()
            out[p + "mask"] = (torch.sigmoid(logits) > 0.5).numpy().astype(np.uint8)
            out[p + "bce"], out[p + "dice"], out[p + "loss"] = lb, ld, loss
            grad_stats(m, p, out)
            out[p + "params_samp"] = param_samples(m)
            bufs = dict(m.named_buffers())
            out[p + "running_mean"] = np.concatenate([bufs[f"{n}.running_mean"].numpy() for n in names])
            out[p + "running_var"] = np.concatenate([bufs[f"{n}.running_var"].numpy() for n in names])
        m.eval()
        with torch.no_grad():
            out[tag + "eval_logits"] = m(x).numpy()
    np.savez_compressed(os.path.join(OUT, "mod_d3_64.npz"), **out)


def case_res_d3_64():
    torch.manual_seed(0)
    m = RefResUNet(1, 1, base_filters=64, depth=3)
    spec = MO.res_param_spec(1, 1, 64, 3)
    assert [n for n, _ in m.named_parameters()] == [s[0] for s in spec], "res param order"
    names = [n for n, _ in MO.res_bn_layers(64, 3)]
    assert [n for n, _ in m.named_buffers() if n.endswith("running_mean")] == \
        [f"{n}.running_mean" for n in names], "res buffer order"
    sd = m.state_dict()
    for k, v in MO.res_make_params(42, 64, 3).items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    m.train()
    x = torch.from_numpy(W.make_input(13, 2, 1, 64, 64))
    t = torch.from_numpy(W.make_target(13, 2, 64, 64))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
    out = {}
    for s in range(2):
        logits, lb, ld, loss = step(m, opt, x, t, RefDice())
        p = f"s{s}_"
        out[p + "logits"] = logits.numpy()
        out[p + "mask"] = (torch.sigmoid(logits) > 0.5).numpy().astype(np.uint8)
        out[p + "bce"], out[p + "dice"], out[p + "loss"] = lb, ld, loss
        grad_stats(m, p, out)
        out[p + "params_samp"] = param_samples(m)
        bufs = dict(m.named_buffers())
        out[p + "running_mean"] = np.concatenate([bufs[f"{n}.running_mean"].numpy() for n in names])
        out[p + "running_var"] = np.concatenate([bufs[f"{n}.running_var"].numpy() for n in names])
    m.eval()
    with torch.no_grad():
        out["eval_logits"] = m(x).numpy()
    np.savez_compressed(os.path.join(OUT, "res_d3_64.npz"), **out)


def case_mod_narrow_64():
    out = {}
    m = build_mod(32, 4)
    m.train()
    x = torch.from_numpy(W.make_input(31, 2, 1, 64, 64))
    t = torch.from_numpy(W.make_target(31, 2, 64, 64))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
    names = [n for n, _ in MO.bn_layers(32, 4)]
    for s in range(2):
        logits, lb, ld, loss = step(m, opt, x, t, RefDice())
        p = f"b32_s{s}_"
        out[p + "logits"] = logits.numpy()
        out[p + "bce"], out[p + "dice"], out[p + "loss"] = lb, ld, loss
        grad_stats(m, p, out)
        out[p + "params_samp"] = param_samples(m)
        bufs = dict(m.named_buffers())
        out[p + "running_mean"] = np.concatenate([bufs[f"{n}.running_mean"].numpy() for n in names])
        out[p + "running_var"] = np.concatenate([bufs[f"{n}.running_var"].numpy() for n in names])
    m.eval()
    with torch.no_grad():
        out["b32_eval_logits"] = m(x).numpy()
    for tag, base in (("u24_", 24), ("u48_", 48)):
        m = build_mod(base, 3)
        m.train()
        logits = m(x)
        lb, ld = torch.nn.BCEWithLogitsLoss()(logits, t), RefDice()(logits, t)
        (lb + ld).backward()
        out[tag + "logits"] = logits.detach().numpy()
        out[tag + "loss"] = (lb + ld).item()
        grad_stats(m, tag, out)
    torch.manual_seed(0)
    m = RefResUNet(1, 1, base_filters=16, depth=3)
    sd = m.state_dict()
    for k, v in MO.res_make_params(42, 16, 3).items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    m.train()
    logits = m(x)
    lb, ld = torch.nn.BCEWithLogitsLoss()(logits, t), RefDice()(logits, t)
    (lb + ld).backward()
    out["r16_logits"] = logits.detach().numpy()
    out["r16_loss"] = (lb + ld).item()
    grad_stats(m, "r16_", out)
    np.savez_compressed(os.path.join(OUT, "mod_narrow_64.npz"), **out)


def _build_res(base, depth, seed=42):
    torch.manual_seed(0)
    m = RefResUNet(1, 1, base_filters=base, depth=depth)
    sd = m.state_dict()
    for k, v in MO.res_make_params(seed, base, depth).items():
        sd[k] = v.clone()
    m.load_state_dict(sd)
    return m


def case_dp_modres_64():
    """nn.DataParallel training of the two networks the reference CLI builds (main.py:122
    ResUNet; models/mod.py:9-66 UNet), base 64, depth 3, B = 3 over two replicas (torch.chunk:
    shards of 2 and 1), BCE + Dice on the gathered logits, gradients summed, two AdamW steps
    (lr 1e-4), then eval with replica 0's buffers (utils/trainer.py:28-30, 81-93, 130)."""
    out = {}
    x = torch.from_numpy(W.make_input(17, 3, 1, 64, 64))
    t = torch.from_numpy(W.make_target(17, 3, 64, 64))
    for tag, m, names in (("res_", _build_res(64, 3), [n for n, _ in MO.res_bn_layers(64, 3)]),
                          ("mod_", build_mod(64, 3), [n for n, _ in MO.bn_layers(64, 3)])):
        m.train()
        opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
        for s in range(2):
            p = f"{tag}s{s}_"
            opt.zero_grad()
            logits = dp_forward(m, x, 2)
            lb = torch.nn.BCEWithLogitsLoss()(logits, t)
            ld = RefDice()(logits, t)
            loss = lb + ld
            loss.backward()
            out[p + "logits"] = logits.detach().numpy()
            out[p + "bce"], out[p + "dice"], out[p + "loss"] = lb.item(), ld.item(), loss.item()
            grad_stats(m, p, out)
            opt.step()
            out[p + "params_samp"] = param_samples(m)
            bufs = dict(m.named_buffers())
            out[p + "running_mean"] = np.concatenate([bufs[f"{n}.running_mean"].numpy() for n in names])
            out[p + "running_var"] = np.concatenate([bufs[f"{n}.running_var"].numpy() for n in names])
        m.eval()
        with torch.no_grad():
            out[tag + "eval_logits"] = m(x).numpy()
    np.savez_compressed(os.path.join(OUT, "modres_dp_64.npz"), **out)


def case_mod_c4_64():
    m = build_mod(128, 5)
    m.train()
    x = torch.from_numpy(W.make_input(12, 2, 1, 64, 64))
    t = torch.from_numpy(W.make_target(12, 2, 64, 64))
    logits = m(x)
    lb = torch.nn.BCEWithLogitsLoss()(logits, t)
    ld = RefDice()(logits, t)
    loss = lb + ld
    loss.backward()
    out = dict(logits=logits.detach().numpy(), bce=lb.item(), dice=ld.item(), loss=loss.item())
    grad_stats(m, "", out)
    np.savez_compressed(os.path.join(OUT, "mod_c4_64.npz"), **out)


if __name__ == "__main__":
    torch.set_num_threads(8)
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[1:]  # optional subset of case names, e.g. focal_64 dp_focal_64
    if only:
        for name in only:
            globals()["case_" + name]()
        sys.exit(0)
    case_b2_64()
    case_b2_256()
    case_dp2_64()
    case_neg_32()
    case_mod_d3_64()
    case_res_d3_64()
    case_mod_c4_64()
    case_focal_64()
    case_dp_focal_64()
    case_mod_narrow_64()
    case_dp_eval_64()
    case_dp_modres_64()
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))
