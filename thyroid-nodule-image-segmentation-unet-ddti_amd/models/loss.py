"""Drop-in for the reference's ``models/loss.py`` on the HIP path.

The three pixel-statistics losses share ONE fused kernel (``unet_hip.seg_losses``):
per-sample sum(p*t), sum(p), sum(t) and the BCE sum are computed in a single pass over
the logits, and each module below just picks its term:

* ``BCEWithLogitsLoss`` - ``nn.BCEWithLogitsLoss()`` mean (utils/trainer.py:37)
* ``DiceLoss``          - soft Dice, per-sample, smooth 1 (models/loss.py:7-24)
* ``FocalTverskyLoss``  - global TP/FP/FN Tversky index ** gamma (models/loss.py:26-46)

``BoundaryLoss`` (models/loss.py:48-66) needs a Euclidean distance transform of each
target on the host (scipy) exactly like the reference; it is off the hot path (its weight
is 0 in every BASELINE config) and is computed with plain torch ops + scipy here.
"""
import numpy as np
import scipy.ndimage as nd
import torch
import torch.nn as nn

from unet_hip import seg_losses


class BCEWithLogitsLoss(nn.Module):
    """Mean binary cross-entropy on logits (``nn.BCEWithLogitsLoss()``), HIP kernel."""

    def forward(self, logits, targets):
        return seg_losses(logits, targets)[0]


class DiceLoss(nn.Module):
    """Soft Dice loss for binary segmentation (reference models/loss.py:7-24)."""

    def __init__(self, smooth=1.0):
        super().__init__()
        if smooth != 1.0:
            raise NotImplementedError("the fused loss kernel implements the reference default smooth=1")
        self.smooth = smooth

    def forward(self, logits, targets):
        return seg_losses(logits, targets)[1]


class FocalTverskyLoss(nn.Module):
    """(1 - TI)^gamma on global TP/FP/FN (reference models/loss.py:26-46)."""

    def __init__(self, alpha=0.4, beta=0.6, gamma=2.0, smooth=1e-6):
        super().__init__()
        if smooth != 1e-6:
            raise NotImplementedError("the fused loss kernel implements the reference default smooth=1e-6")
        self.alpha, self.beta, self.gamma, self.smooth = alpha, beta, gamma, smooth

    def forward(self, logits, targets):
        return seg_losses(logits, targets, self.alpha, self.beta, self.gamma)[2]


def _distance_maps(targets):
    """EDT of the background of each (binarised) target, float32 (N, 1, H, W) on targets' device."""
    t = targets.detach().cpu().numpy().astype(np.uint8)
    out = np.stack([nd.distance_transform_edt(1 - t[b, 0]) for b in range(t.shape[0])])
    return torch.from_numpy(out[:, None].astype(np.float32)).to(targets.device)


class BoundaryLoss(nn.Module):
    """mean_b mean_hw |sigmoid(x) - t| * EDT(1 - t)   (reference models/loss.py:48-66)."""

    def forward(self, logits, targets):
        dist = _distance_maps(targets)
        per = (torch.abs(torch.sigmoid(logits) - targets) * dist).flatten(1).mean(1)
        return per.mean()


class CompositeLoss(nn.Module):
    """λ_ft·FocalTversky(0.3, 0.7, 0.75) + λ_b·Boundary [+ λ_bce·BCE + λ_dice·Dice]
    (reference models/loss.py:68-82)."""

    def __init__(self, λ_ft=1.0, λ_b=0.5, λ_bce=0.0, λ_dice=0.0):
        super().__init__()
        self.λ_ft, self.λ_b, self.λ_bce, self.λ_dice = λ_ft, λ_b, λ_bce, λ_dice
        self.bl = BoundaryLoss()

    def forward(self, logits, targets):
        l = seg_losses(logits, targets, 0.3, 0.7, 0.75)
        loss = self.λ_ft * l[2] + self.λ_b * self.bl(logits, targets)
        if self.λ_bce > 0:
            loss = loss + self.λ_bce * l[0]
        if self.λ_dice > 0:
            loss = loss + self.λ_dice * l[1]
        return loss
