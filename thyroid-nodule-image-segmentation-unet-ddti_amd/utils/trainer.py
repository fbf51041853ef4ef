"""Trainer for the HIP UNet path (mirror of the reference's utils/trainer.py).

Same constructor ``Trainer(config, (train, val, test loaders), logger, model)`` and the same
``train / train_one_epoch / validate / test`` flow as the reference (utils/trainer.py:19-299):
AdamW(lr) with torch-default betas/eps/weight-decay (:41), CosineAnnealingWarmRestarts(20, 2)
(:42), early stopping on -val IoU (:44,194-197), best/last checkpoints of the bare
state_dict (:184-202), mixup (:62-78), loss = bce_ratio*BCE + dice_ratio*Dice +
focal_ratio*FocalTversky + boundary_ratio*Boundary (:85-90).

What runs where (MI355X-first):
* forward / backward: libunet_hip.so via ``models.model.UNet``;
* BCE + Dice + FocalTversky: ONE fused HIP statistics kernel per step and ONE dlogits
  kernel in backward (weights = the ratios, no host sync);
* optimizer: ``HipAdamW`` (one native launch over the flat 31M-float arena);
* metrics: masks and confusion counts on the device (``unet_mask_counts``); only 6
  integers per step come back instead of the reference's full prediction arrays (the
  epoch metrics are sums of those counts, so the numbers are the same);
* multi-GPU: one process per GPU (``torch.distributed`` with the "nccl" = RCCL backend
  initialised by the launcher) with bucketed gradient all-reduce overlapped with the
  backward, replacing ``nn.DataParallel`` (:28-30).  Every rank takes its torch.chunk share
  of each global batch (data.data_loader.DataParallelShardSampler, ``--batch_size`` stays
  global), runs per-rank BatchNorm as DataParallel's replicas do, gets the gathered batch's
  losses (incl. FocalTversky's global TP/FP/FN) and the summed gradients; epoch meters and
  confusion counts are summed over ranks.
* BoundaryLoss keeps the reference's host EDT and is only evaluated when its ratio != 0
  (the reference evaluates it every step even at ratio 0; 0 * finite == 0, so skipping it
  changes no number).
"""
import os
import random

import numpy as np
import torch
import torch.distributed as dist
from torch.optim.lr_scheduler import CosineAnnealingWarmRestarts

import unet_hip
from models.loss import BoundaryLoss
from unet_hip.dist import DistributedUNet
from utils.utils import AverageMeter, EarlyStopping, global_metrics_from_counts, metrics_from_counts

try:
    from torch.utils.tensorboard import SummaryWriter
except Exception:  # tensorboard is not installed in every image: logging only
    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

        def close(self):
            pass

class _NullWriter:
    def add_scalar(self, *a, **k):
        pass

    def close(self):
        pass


try:
    from tqdm import tqdm
except Exception:
    def tqdm(it, **k):
        return it


def _distributed():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _is_rank0():
    return not _distributed() or dist.get_rank() == 0


class _Rank0Logger:
    """Under data parallelism every rank runs the Trainer, but the reference's single process
    writes each log line once: only rank 0 forwards to the shared logger (whose file handler
    all ranks would otherwise append to)."""

    def __init__(self, logger, enabled):
        self._logger, self._enabled = logger, enabled

    def __getattr__(self, name):
        attr = getattr(self._logger, name)
        if name in ("debug", "info", "warning", "error", "critical", "exception", "log") \
                and not self._enabled:
            return lambda *a, **k: None
        return attr


class Trainer:
    def __init__(self, config, data_loader, logger, model):
        self.config = config
        self.rank0 = _is_rank0()
        self.logger = _Rank0Logger(logger, self.rank0)
        dev = getattr(config, "device", torch.device("cuda"))
        if _distributed():
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.train_loader, self.val_loader, self.test_loader = data_loader
        self.model = model.to(self.device)
        self.model.flatten_()
        self.optimizer = unet_hip.HipAdamW(self.model.parameters(), lr=config.lr)
        self.ddp = None
        if _distributed():
            self.logger.info(f"Using {dist.get_world_size()} GPUs (one process each, RCCL)")
            self.ddp = DistributedUNet(self.model, self.optimizer)
        self.scheduler = CosineAnnealingWarmRestarts(self.optimizer, T_0=20, T_mult=2, eta_min=0)
        self.focal_abg = (0.4, 0.6, 2.0)  # FocalTverskyLoss() defaults (utils/trainer.py:38)
        self.criterion_boundary = BoundaryLoss()
        self.early_stopping = EarlyStopping(logger=self.logger,
                                            patience=getattr(config, "early_stop_patience", 50), delta=0)
        self.writer = (SummaryWriter(log_dir=getattr(config, "result_dir", None)) if self.rank0
                       else _NullWriter())
        self.rt = self.model._state.rt

    # -------------------------------------------------------------- helpers
    def _losses(self, logits, masks):
        """-> (loss to differentiate, [bce, dice, focal], boundary, reported total).  Under
        data parallelism the first is this rank's share of the gathered batch's loss (its
        gradient summed over the ranks is DataParallel's), the others are the gathered
        batch's values (same on every rank)."""
        c = self.config
        if self.ddp is not None:  # the gathered batch's losses (nn.DataParallel semantics)
            l = self.ddp.losses(logits, masks, *self.focal_abg)
        else:
            l = unet_hip.seg_losses(logits, masks, *self.focal_abg)
        w = torch.tensor([c.bce_ratio, c.dice_ratio, c.focal_ratio], device=logits.device)
        loss = (w * l).sum()
        lb = torch.zeros((), device=logits.device)
        total = loss
        if c.boundary_ratio != 0:
            lb = self.criterion_boundary(logits, masks)  # mean over this rank's samples
            if self.ddp is not None:
                # gathered-batch mean (models/loss.py:66 divides by the full batch): weight
                # the local mean by n_local / n_global; gradients are summed over ranks
                n = torch.tensor([float(logits.shape[0])], device=logits.device)
                dist.all_reduce(n)
                lb = lb * (logits.shape[0] / float(n.item()))
                loss = loss + c.boundary_ratio * lb
                lb = lb.detach().clone()
                dist.all_reduce(lb)
                total = total.detach() + c.boundary_ratio * lb
            else:
                loss = loss + c.boundary_ratio * lb
                total = loss
        return loss, l, lb, total

    def _rank0_mixup(self, mix, lam):
        d = torch.tensor([1.0 if mix else 0.0, lam if mix else 0.0], dtype=torch.float64,
                         device=self.device)
        dist.broadcast(d, src=self.ddp._src(), group=self.ddp.group)
        mix = bool(d[0].item() != 0.0)
        return mix, (float(d[1].item()) if mix else None)

    def _reduce_scalars(self, sums, n_seen):
        """Epoch means weighted like the reference's AverageMeter.update(loss, batch size)
        over the gathered batches: sum Σ(l·b) and Σb over the ranks, then divide."""
        v = torch.cat([sums, torch.tensor([float(n_seen)], dtype=sums.dtype, device=sums.device)])
        if _distributed():
            dist.all_reduce(v)
        n = max(float(v[-1]), 1.0)
        return v[:-1] / n, n

    def _reduce_counts(self, c):
        if _distributed():
            dist.all_reduce(c)
        return c

    def _log_epoch(self, tag, epoch, meters, counts):
        acc, precision, recall, f1, iou = metrics_from_counts(counts.tolist())
        bce, dice, focal, bnd, tot = (m.avg for m in meters)
        self.logger.info(f"{tag} Epoch: {epoch + 1}, Avg Loss: {tot:.4f}")
        self.logger.info(f"BCE Loss: {bce:.4f}, Dice Loss: {dice:.4f}, Focal Loss: {focal:.4f}, "
                         f"Boundary Loss: {bnd:.4f}")
        self.logger.info(f"acc: {acc:.4f}, precision: {precision:.4f}, recall: {recall:.4f}, "
                         f"f1: {f1:.4f}, IoU: {iou:.4f}")
        name = "Train" if tag == "Train" else "Validate"
        for k, v in (("BCE Loss", bce), ("Dice Loss", dice), ("Focal Loss", focal),
                     ("Boundary Loss", bnd), ("Acc", acc), ("Precision", precision),
                     ("Recall", recall), ("F1", f1), ("IoU", iou)):
            self.writer.add_scalar(f"{k}/{name}", v, epoch)
        return iou

    def _run_epoch(self, loader, epoch, train):
        meters = [AverageMeter() for _ in range(5)]
        counts = torch.zeros(6, dtype=torch.int64, device=self.device)
        sums = torch.zeros(5, dtype=torch.float64, device=self.device)  # device-side meters
        n_seen = 0
        desc = f"{'Training' if train else 'Validating'} Epoch {epoch + 1}"
        bsamp = getattr(loader, "batch_sampler", None)
        if hasattr(bsamp, "set_epoch"):  # DataParallelShardSampler: same batches on every rank
            bsamp.set_epoch(epoch)
        nb_extra = 2 if self.config.boundary_ratio != 0 else 0
        for batch in tqdm(loader, desc=desc, leave=True):
            # utils/trainer.py:62-78: the mixup draws (random, numpy beta, then a CPU
            # torch.randperm of the batch size) come first and are consumed alike on every
            # rank (ranks share the seeds, set_seed(42)), even when a rank's shard is empty.
            # Under data parallelism the GATHERED batch is mixed, as the reference mixes the
            # whole batch before DataParallel scatters it, and each rank keeps its slice.
            mix = train and random.random() < self.config.mixup_prob and self.config.use_mixup
            lam = np.random.beta(self.config.mixup_alpha, self.config.mixup_alpha) if mix else None
            if train and self.config.use_mixup and self.ddp is not None:
                # the host RNG streams differ per rank (per-rank augmentation seeds, shards of
                # unequal size), but gather_batch is a collective: rank 0's draws decide
                mix, lam = self._rank0_mixup(mix, lam)
            if batch is not None:
                images, masks = batch
                images = images.to(self.device, non_blocking=True).float()
                masks = masks.to(self.device, non_blocking=True).float()
            if mix and self.ddp is not None:
                gi, gm, off, n = self.ddp.gather_batch(None if batch is None else images,
                                                       None if batch is None else masks, self.device)
                perm = torch.randperm(gi.size(0)).to(self.device)
                dist.broadcast(perm, src=self.ddp._src(), group=self.ddp.group)
                if batch is not None:
                    sl = slice(off, off + n)
                    images = lam * gi[sl] + (1.0 - lam) * gi[perm[sl]]
                    masks = lam * gm[sl] + (1.0 - lam) * gm[perm[sl]]
            elif mix:
                perm = torch.randperm(images.size(0)).to(self.device)
                images = lam * images + (1.0 - lam) * images[perm]
                masks = lam * masks + (1.0 - lam) * masks[perm]
            if batch is None:  # empty DataParallel shard: join the step's collectives only
                if train:
                    self.optimizer.zero_grad(set_to_none=True)
                    self.ddp.empty_step(nb_extra)
                    self.optimizer.step()
                else:
                    self.ddp.empty_losses(nb_extra)
                continue
            if train:
                self.optimizer.zero_grad(set_to_none=True)
                logits = self.model(images)
                loss, l, lb, total = self._losses(logits, masks)
                loss.backward()
                if self.ddp is not None:
                    self.ddp.reduce_gradients()
                self.optimizer.step()
            else:
                with torch.no_grad():
                    logits = self.model(images)
                    loss, l, lb, total = self._losses(logits, masks)
            bs = masks.size(0)
            sums += torch.stack([l[0], l[1], l[2], lb, total]).detach().double() * bs
            n_seen += bs
            self.rt.mask_counts(logits.detach(), masks, counts)
        totals, n_glob = self._reduce_scalars(sums, n_seen)
        for m, v in zip(meters, totals.tolist()):
            m.update(v, n_glob)  # the global count: identical meters on every rank
        return meters, self._reduce_counts(counts)

    # -------------------------------------------------------------- reference API
    def train_one_epoch(self, epoch):
        self.model.train()
        meters, counts = self._run_epoch(self.train_loader, epoch, True)
        self._log_epoch("Train", epoch, meters, counts)
        return meters[4].avg

    @torch.no_grad()
    def validate(self, epoch):
        self.model.eval()
        if self.ddp is not None:  # every shard evaluated with replica 0's BN buffers (DataParallel)
            self.ddp.sync_buffers()
        meters, counts = self._run_epoch(self.val_loader, epoch, False)
        iou = self._log_epoch("Validate", epoch, meters, counts)
        return meters[4].avg, iou

    def _save(self, path):
        if not _distributed() or dist.get_rank() == 0:
            torch.save({k: v.detach().clone().cpu() for k, v in self.model.state_dict().items()}, path)

    def train(self):
        best_val_iou = -np.inf
        mt = getattr(self.config, "model_type", "UNet")
        for epoch in range(self.config.epochs):
            self.train_one_epoch(epoch)
            val_loss, val_iou = self.validate(epoch)
            self.scheduler.step()
            if val_iou > best_val_iou:
                best_val_iou = val_iou
                self._save(os.path.join(self.config.model_dir, f"{mt}_best.pth"))
                self.logger.info(f"--Best model saved at epoch {epoch + 1} with IoU: {best_val_iou:.4f}")
            self.early_stopping(-val_iou, self)
            if self.early_stopping.early_stop:
                self.logger.info("--Early stopping triggered")
                break
        self._save(os.path.join(self.config.model_dir, f"{mt}_last.pth"))
        self.writer.close()

    @torch.no_grad()
    def test(self):
        """Global pixel TP/FP/FN/TN over the test set (utils/trainer.py:206-260); counts are
        accumulated on the device.  The contour-overlay PNGs (:262-299) are written only when
        matplotlib and scikit-image are importable."""
        self.logger.info("------------------Starting Testing Model------------------")
        self.model.eval()
        if self.ddp is not None:  # every shard evaluated with replica 0's BN buffers (DataParallel)
            self.ddp.sync_buffers()
        counts = torch.zeros(6, dtype=torch.int64, device=self.device)
        total = 0
        keep = []
        for batch in tqdm(self.test_loader, desc="Testing Model", leave=True):
            if batch is None:  # empty DataParallel shard: nothing to count on this rank
                keep.append(None)
                continue
            images, masks = batch
            images = images.to(self.device).float()
            masks = masks.to(self.device).float()
            logits = self.model(images)
            mask = torch.empty(logits.shape, dtype=torch.uint8, device=self.device)
            self.rt.mask_counts(logits, masks, counts, mask)
            total += images.size(0)
            keep.append((images.cpu(), masks.cpu(), mask.cpu()))
        if _distributed():
            nt = torch.tensor([total], dtype=torch.int64, device=self.device)
            dist.all_reduce(nt)
            total = int(nt.item())
        m = global_metrics_from_counts(self._reduce_counts(counts).tolist())
        msg = (f"Test Metrics  —  Total Images: {total}\n"
               f"  TP={m['TP']}, FP={m['FP']}, FN={m['FN']}, TN={m['TN']}\n"
               f"  ACC={m['ACC']:.4f}, Precision={m['Precision']:.4f}, "
               f"Recall={m['Recall']:.4f}, F1={m['F1']:.4f}, IoU={m['IoU']:.4f}")
        if self.rank0:
            print(msg)
        self.logger.info(msg)
        if _distributed() and self._can_plot():
            # one set of PNGs over the whole test set, in the reference's sample order: batch
            # by batch, each batch's shards in rank order (DataParallel's gather order)
            # (gather to rank 0 only: it alone plots, so the other ranks need no copies)
            parts = [None] * dist.get_world_size() if self.rank0 else None
            dist.gather_object(keep, parts, dst=0)
            keep = ([p[b] for b in range(len(parts[0])) for p in parts if b < len(p)]
                    if self.rank0 else [])
        keep = [k for k in keep if k is not None]
        if keep and self.rank0:
            self._plot_contours(keep)
        return m

    @staticmethod
    def _can_plot():
        try:
            import matplotlib  # noqa: F401
            from skimage import measure  # noqa: F401
        except Exception:
            return False
        return True

    def _plot_contours(self, keep):
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
            from skimage import measure
        except Exception:
            self.logger.info("contour plots skipped (matplotlib / scikit-image not available)")
            return
        imgs = torch.cat([k[0] for k in keep]).numpy()
        gts = torch.cat([k[1] for k in keep]).numpy().astype(np.uint8)
        prs = torch.cat([k[2] for k in keep]).numpy()
        for start in range(0, len(imgs), 20):
            fig, axes = plt.subplots(5, 4, figsize=(16, 20))
            axes = axes.flatten()
            for i, idx in enumerate(range(start, min(start + 20, len(imgs)))):
                ax = axes[i]
                ax.imshow(imgs[idx].transpose(1, 2, 0).squeeze(), cmap="gray")
                for c in measure.find_contours(gts[idx].squeeze(), level=0.5):
                    ax.plot(c[:, 1], c[:, 0], color="blue", linewidth=1)
                for c in measure.find_contours(prs[idx].squeeze(), level=0.5):
                    ax.plot(c[:, 1], c[:, 0], color="red", linewidth=1)
            for ax in axes:
                ax.axis("off")
            plt.tight_layout()
            plt.savefig(os.path.join(self.config.result_dir, f"test_boundaries_{start // 20}.png"))
            plt.close(fig)
