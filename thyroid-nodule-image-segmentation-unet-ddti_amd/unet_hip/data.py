"""Device-side input pipeline: the reference's Resize + ToTensor (utils/transforms.py:
143-156, applied per sample by data/data_loader.py:20-27) on the GPU.

The reference resizes every image AND mask with ``TF.resize`` -- for PIL images that is
Pillow's ``Image.resize(size, BILINEAR)`` (masks too: they become soft targets) -- and
then ``TF.to_tensor`` = float(u8) / 255.  Here the host only decodes (JPEG -> uint8), the
uint8 planes travel to HBM (1 B/pixel instead of 4), and ``unet_resize_u8`` produces the
fp32 batch directly, bit-identical to Pillow (tests/test_gpu_data.py).

    pipe = GpuResizeToTensor((512, 512), device="cuda")
    x, t = pipe(images, masks)           # lists of HxW uint8 arrays / tensors (any sizes)
                                         # -> (N, 1, 512, 512) fp32 each, on the device

Palette ("P") and bilevel ("1") images: Pillow's Image.resize switches to NEAREST for
those modes whatever filter is asked for.  Planes tagged ``resample="nearest"``
(data.data_loader.DecodeU8 does that) run the same kernel with a one-tap plan: source
index = int(x0), x0 = s/2 then += s per output pixel (s = in/out, Pillow's accumulated
double coordinate of ImagingScaleAffine), coefficient 1.0 in 22-bit fixed point.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .runtime import UNetRuntime


def resize_plan(in_size, out_size):
    """Pillow's coefficients (int32 [out, ksize]) and bounds (int32 [out, 2]) for one axis."""
    lib = _lib.load()
    ks = ctypes.c_int()
    _lib.check(lib.unet_resize_plan(in_size, out_size, None, None, ctypes.byref(ks)), None,
               "unet_resize_plan")
    k = np.zeros((out_size, ks.value), np.int32)
    b = np.zeros((out_size, 2), np.int32)
    _lib.check(lib.unet_resize_plan(in_size, out_size, k.ctypes.data, b.ctypes.data,
                                    ctypes.byref(ks)), None, "unet_resize_plan")
    return k, b


def nearest_plan(in_size, out_size):
    """One-tap plan reproducing Pillow's NEAREST scale (coefficient 1 << 22 at the nearest
    source index)."""
    k = np.full((out_size, 1), 1 << 22, np.int32)
    b = np.ones((out_size, 2), np.int32)
    step = float(in_size) / out_size
    xo = step * 0.5
    for x in range(out_size):
        b[x, 0] = min(int(xo), in_size - 1)
        xo += step
    return k, b


class GpuResizeToTensor:
    """Batched Resize((H, W)) + ToTensor of (image, mask) pairs on the device."""

    def __init__(self, size, device="cuda"):
        self.oh, self.ow = (size, size) if isinstance(size, int) else tuple(size)
        self.device = torch.device(device)
        self.rt = UNetRuntime.get(self.device)
        self._plans = {}

    def _plan(self, n_in, n_out, nearest=False):
        key = (n_in, n_out, nearest)
        if key not in self._plans:
            k, b = nearest_plan(n_in, n_out) if nearest else resize_plan(n_in, n_out)
            self._plans[key] = (torch.from_numpy(k).to(self.device),
                                torch.from_numpy(b).to(self.device), k.shape[1])
        return self._plans[key]

    def resize(self, img, out=None):
        """One HxW uint8 image -> (oh, ow) fp32 in [0, 1] on the device."""
        nearest = getattr(img, "resample", "bilinear") == "nearest"
        if isinstance(img, np.ndarray):  # PIL-backed arrays are read-only views
            img = np.require(img, requirements=["C", "W"])
        t = torch.as_tensor(img)
        if t.dtype != torch.uint8 or t.dim() != 2:
            raise ValueError("expected an (H, W) uint8 image (decoded 'L' mode)")
        t = t.to(self.device, non_blocking=True).contiguous()
        h, w = t.shape
        if out is None:
            out = torch.empty((self.oh, self.ow), dtype=torch.float32, device=self.device)
        kh, bh, ksh = self._plan(w, self.ow, nearest)
        kv, bv, ksv = self._plan(h, self.oh, nearest)
        _lib.check(self.rt.lib.unet_resize_u8(
            self.rt.ctx, _lib.ptr(t), h, w, _lib.ptr(out), self.oh, self.ow, _lib.ptr(kh),
            _lib.ptr(bh), ksh, _lib.ptr(kv), _lib.ptr(bv), ksv, 255.0,
            _lib.stream_ptr(self.device)), self.rt.ctx, "unet_resize_u8")
        return out

    def __call__(self, images, masks=None):
        n = len(images)
        x = torch.empty((n, 1, self.oh, self.ow), dtype=torch.float32, device=self.device)
        for i, im in enumerate(images):
            self.resize(im, x[i, 0])
        if masks is None:
            return x
        t = torch.empty_like(x)
        for i, m in enumerate(masks):
            self.resize(m, t[i, 0])
        return x, t
