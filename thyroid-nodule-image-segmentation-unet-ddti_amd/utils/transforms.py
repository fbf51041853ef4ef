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


def _to_tensor(pic):
    """torchvision TF.to_tensor for a PIL image (utils/transforms.py:152-156 calls it on
    both the image and the mask): the image's OWN mode is kept -- (C, H, W) with C = the
    mode's bands ("L" 1, "RGB" 3, ...); 8-bit data is divided by 255 (torch division),
    mode "1" becomes {0, 1}; 16/32-bit integer and float modes are returned unscaled."""
    nptype = {"I": np.int32, "I;16": np.int16, "F": np.float32}.get(pic.mode, np.uint8)
    a = np.array(pic, dtype=nptype, copy=True)
    if pic.mode == "1":
        a = 255 * a.astype(np.uint8)
    t = torch.from_numpy(a)
    t = t.view(pic.size[1], pic.size[0], -1).permute(2, 0, 1).contiguous()
    if t.dtype == torch.uint8:
        return t.to(torch.float32).div(255)
    return t


class ToTensor:
    """PIL -> tensors exactly as the reference's ToTensor (TF.to_tensor of each)."""

    def __call__(self, img, mask):
        return _to_tensor(img), _to_tensor(mask)


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
