"""Paired (image, mask) transforms used by main.py (subset of the reference's
utils/transforms.py).  ``Compose``, ``Resize`` and ``ToTensor`` behave like the
reference's (:143-165: ``TF.resize`` of both PIL images = Pillow BILINEAR, the mask
included; [0, 1] float tensors).  ``unet_hip.GpuResizeToTensor`` does the same two steps
on the device, bit-identically.  The ultrasound
augmentations (Elastic, Speckle, TGC, CLAHE, Rotate, Flip, Brightness; :15-141) need
OpenCV / torchvision, which are not part of this image, and are host-side data
augmentation outside the accelerated path: constructing them raises NotImplementedError.
"""
import numpy as np
import torch


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, img, mask):
        for t in self.transforms:
            img, mask = t(img, mask)
        return img, mask


class Resize:
    def __init__(self, size):
        self.size = tuple(size)

    def __call__(self, img, mask):
        from PIL import Image
        h, w = self.size
        # TF.resize's default interpolation is BILINEAR for the mask too (soft targets)
        return img.resize((w, h), Image.BILINEAR), mask.resize((w, h), Image.BILINEAR)


class ToTensor:
    """PIL -> float tensors in [0, 1]: image (C, H, W) grayscale, mask (1, H, W)."""

    def __call__(self, img, mask):
        a = np.asarray(img.convert("L"), dtype=np.float32) / 255.0
        m = np.asarray(mask.convert("L"), dtype=np.float32) / 255.0
        return torch.from_numpy(a[None].copy()), torch.from_numpy(m[None].copy())


def _unavailable(name):
    class _T:
        def __init__(self, *a, **k):
            raise NotImplementedError(f"{name} (host augmentation) is not provided on this path")
    _T.__name__ = name
    return _T


ElasticDeform = _unavailable("ElasticDeform")
SpeckleNoise = _unavailable("SpeckleNoise")
TGCAugment = _unavailable("TGCAugment")
CLAHE = _unavailable("CLAHE")
Flip = _unavailable("Flip")
Rotate = _unavailable("Rotate")
AdjustBrightness = _unavailable("AdjustBrightness")
