"""Restatement of Pillow's 8-bit BILINEAR resampler (test infra only).

The reference's Resize (utils/transforms.py:143-149) calls torchvision ``TF.resize`` on PIL
images, which is Pillow ``Image.resize(size, Image.BILINEAR)`` (Pillow 12.2.0 here,
libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc,
ImagingResampleHorizontal_8bpc / Vertical_8bpc): separable triangle filter whose support
scales with the reduction factor, coefficients in 22-bit fixed point, rounding bias
2**21, clip to uint8 after each pass, horizontal pass first.  ToTensor (:151-156) is
float(u8) / 255.  Pillow itself (importable here and on the GPU box) is the ground truth
these functions are checked against in tests/test_data_cpu.py.
"""
import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def plan(in_size, out_size):
    """(coeffs int32 [out, ksize], bounds int32 [out, 2]) exactly as precompute_coeffs +
    normalize_coeffs_8bpc for the full extent [0, in_size)."""
    scale = filterscale = float(in_size) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    kk = np.zeros((out_size, ksize), np.int32)
    bounds = np.zeros((out_size, 2), np.int32)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = []
        ww = 0.0
        for x in range(xmax):
            a = abs((x + xmin - center + 0.5) * ss)
            w = 1.0 - a if a < 1.0 else 0.0
            k.append(w)
            ww += w
        if ww != 0.0:
            k = [v / ww for v in k]
        for x, v in enumerate(k):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return kk, bounds


def _pass(a, kk, bounds):
    """Resample axis 1 of a (rows, in) uint8 array."""
    out = np.empty((a.shape[0], kk.shape[0]), np.uint8)
    for xx in range(kk.shape[0]):
        xmin, n = bounds[xx]
        ss = (1 << (PRECISION_BITS - 1)) + a[:, xmin:xmin + n].astype(np.int64) @ kk[xx, :n].astype(np.int64)
        out[:, xx] = np.clip(ss >> PRECISION_BITS, 0, 255)
    return out


def resize_u8(img, oh, ow):
    """uint8 (h, w) -> uint8 (oh, ow), Pillow BILINEAR."""
    a = np.asarray(img, np.uint8)
    if a.shape[1] != ow:
        a = _pass(a, *plan(a.shape[1], ow))
    if a.shape[0] != oh:
        a = _pass(a.T, *plan(a.shape[0], oh)).T
    return np.ascontiguousarray(a)


def nearest_index(in_size, out_size):
    """Pillow's NEAREST scale (Image.resize forces it for "P" and "1" images; libImaging
    Geometry.c ImagingScaleAffine): the source coordinate starts at s/2, s = in/out, and
    is advanced by += s in double per output pixel; index = int(coordinate)."""
    s = float(in_size) / out_size
    xo = s * 0.5
    idx = np.empty(out_size, np.int64)
    for x in range(out_size):
        idx[x] = int(xo)
        xo += s
    return idx


def resize_nearest_u8(img, oh, ow):
    a = np.asarray(img, np.uint8)
    return np.ascontiguousarray(a[nearest_index(a.shape[0], oh)][:, nearest_index(a.shape[1], ow)])


def to_tensor(img_u8):
    """TF.to_tensor of an 'L' image: float32(u8) / 255."""
    return np.asarray(img_u8, np.float32) / np.float32(255.0)
