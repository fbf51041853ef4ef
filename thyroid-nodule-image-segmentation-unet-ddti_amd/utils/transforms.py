"""Paired (image, mask) transforms of the reference's utils/transforms.py.

Host-side data preparation in front of the accelerated path (PIL images in, before
``Resize`` + ``ToTensor`` -- or before ``DecodeU8`` when the resize runs on the GPU,
``unet_hip.GpuResizeToTensor``, bit-identically).  Every class draws from Python's
``random`` and NumPy's global RNG in the same order and with the same calls as the
reference, so a seeded run (``utils.utils.set_seed``) takes the same augmentation
decisions and parameters.

torchvision and OpenCV are not in this image, so the library calls are restated:
  * ``Flip`` / ``Rotate`` / ``AdjustBrightness`` / ``RandomCrop`` / ``Resize`` /
    ``ToTensor`` (:84-156): torchvision's PIL kernels are single Pillow calls
    (``TF.hflip`` = ``Image.transpose``, ``TF.rotate`` = ``Image.rotate`` with NEAREST and
    fill 0, ``TF.adjust_brightness`` = ``ImageEnhance.Brightness``, ``TF.crop`` =
    ``Image.crop``, ``TF.resize`` = ``Image.resize`` BILINEAR), made here directly: the
    same pixels;
  * ``SpeckleNoise`` / ``TGCAugment`` (:44-70) are NumPy in the reference and here;
  * ``ElasticDeform`` (:14-42) and ``CLAHE`` (:72-81) restate ``cv2.GaussianBlur`` +
    ``cv2.remap`` and ``cv2.createCLAHE`` in NumPy from OpenCV's algorithms (separable
    double-precision Gaussian with BORDER_REFLECT_101; remap on 1/32-pixel fixed-point
    coordinates with 15-bit integer bilinear weights, BORDER_REFLECT; CLAHE's clipped tile
    histograms and bilinear LUT interpolation in float32).  Parity unpinned: there is no
    OpenCV here to compare with (tests/test_transforms_cpu.py checks their invariants).
"""
import random

import numpy as np
import torch
from PIL import Image, ImageEnhance


# ---------------------------------------------------------------------------------------
# OpenCV restatements (ElasticDeform, CLAHE)
# ---------------------------------------------------------------------------------------
def gaussian_kernel(ksize, sigma):
    """cv2.getGaussianKernel(ksize, sigma, CV_64F) for sigma > 0."""
    x = np.arange(ksize, dtype=np.float64) - (ksize - 1) * 0.5
    k = np.exp(-(x * x) / (2.0 * sigma * sigma))
    return k / k.sum()


def gaussian_blur(a, ksize, sigma):
    """cv2.GaussianBlur(a (float64 2-D), (ksize, ksize), sigmaX=sigma): separable, rows
    first, BORDER_REFLECT_101 (numpy's "reflect")."""
    k = gaussian_kernel(ksize, sigma)
    r = ksize // 2
    h, w = a.shape
    p = np.pad(np.asarray(a, np.float64), r, mode="reflect")
    t = np.zeros((h + 2 * r, w), np.float64)
    for i in range(ksize):
        t += k[i] * p[:, i:i + w]
    out = np.zeros((h, w), np.float64)
    for i in range(ksize):
        out += k[i] * t[i:i + h, :]
    return out


def _reflect(i, n):
    """cv2.borderInterpolate(i, n, BORDER_REFLECT): fedcba|abcdefgh|hgfedcb."""
    if n == 1:
        return np.zeros_like(i)
    period = 2 * n
    i = np.mod(i, period)
    return np.where(i >= n, period - 1 - i, i)


def remap_linear_u8(src, map_x, map_y):
    """cv2.remap(src uint8 2-D, map_x, map_y (float32), INTER_LINEAR, BORDER_REFLECT):
    coordinates rounded to 1/32 pixel, integer weights (32 - fx)(32 - fy) * 32 etc. summing
    to 2^15, result (sum + 2^14) >> 15."""
    h, w = src.shape
    X = np.rint(map_x.astype(np.float32) * np.float32(32)).astype(np.int64)
    Y = np.rint(map_y.astype(np.float32) * np.float32(32)).astype(np.int64)
    x0, y0 = X >> 5, Y >> 5
    fx, fy = X & 31, Y & 31
    xs0, xs1 = _reflect(x0, w), _reflect(x0 + 1, w)
    ys0, ys1 = _reflect(y0, h), _reflect(y0 + 1, h)
    s = src.astype(np.int64)
    v = (s[ys0, xs0] * ((32 - fx) * (32 - fy)) + s[ys0, xs1] * (fx * (32 - fy)) +
         s[ys1, xs0] * ((32 - fx) * fy) + s[ys1, xs1] * (fx * fy)) * 32
    return np.clip((v + (1 << 14)) >> 15, 0, 255).astype(np.uint8)


def remap_nearest(src, map_x, map_y):
    """cv2.remap(..., INTER_NEAREST, BORDER_REFLECT): cvRound of each coordinate."""
    h, w = src.shape[:2]
    xi = np.rint(map_x.astype(np.float32)).astype(np.int64)
    yi = np.rint(map_y.astype(np.float32)).astype(np.int64)
    return src[_reflect(yi, h), _reflect(xi, w)]


def clahe_u8(img, clip=2.0, grid=(4, 4)):
    """cv2.createCLAHE(clipLimit=clip, tileGridSize=grid).apply(img uint8 2-D)."""
    h, w = img.shape
    tx, ty = grid
    ext = img
    if w % tx or h % ty:  # cv2 pads bottom/right with BORDER_REFLECT_101 to whole tiles
        ext = np.pad(img, ((0, ty - h % ty if h % ty else 0), (0, tx - w % tx if w % tx else 0)),
                     mode="reflect")
    th, tw = ext.shape[0] // ty, ext.shape[1] // tx
    area = th * tw
    lut_scale = np.float32(255.0 / area)
    limit = max(int(clip * area / 256), 1) if clip > 0 else 0
    lut = np.zeros((ty, tx, 256), np.uint8)
    for j in range(ty):
        for i in range(tx):
            hist = np.bincount(ext[j * th:(j + 1) * th, i * tw:(i + 1) * tw].ravel(),
                               minlength=256).astype(np.int64)
            if limit > 0:
                clipped = int(np.maximum(hist - limit, 0).sum())
                hist = np.minimum(hist, limit)
                batch = clipped // 256
                residual = clipped - batch * 256
                hist += batch
                if residual:
                    step = max(256 // residual, 1)
                    k = 0
                    while k < 256 and residual > 0:
                        hist[k] += 1
                        k += step
                        residual -= 1
            cum = np.cumsum(hist).astype(np.float32)
            lut[j, i] = np.clip(np.rint(cum * lut_scale), 0, 255).astype(np.uint8)
    inv_tw, inv_th = np.float32(1.0) / np.float32(tw), np.float32(1.0) / np.float32(th)
    txf = np.arange(w, dtype=np.float32) * inv_tw - np.float32(0.5)
    tx1 = np.floor(txf).astype(np.int64)
    xa = (txf - tx1.astype(np.float32)).astype(np.float32)
    xa1 = np.float32(1.0) - xa
    tx2 = np.minimum(tx1 + 1, tx - 1)
    tx1 = np.maximum(tx1, 0)
    tyf = np.arange(h, dtype=np.float32) * inv_th - np.float32(0.5)
    ty1 = np.floor(tyf).astype(np.int64)
    ya = (tyf - ty1.astype(np.float32)).astype(np.float32)[:, None]
    ya1 = np.float32(1.0) - ya
    ty2 = np.minimum(ty1 + 1, ty - 1)[:, None]
    ty1 = np.maximum(ty1, 0)[:, None]
    v = img.astype(np.int64)
    l11 = lut[ty1, tx1[None, :], v].astype(np.float32)
    l12 = lut[ty1, tx2[None, :], v].astype(np.float32)
    l21 = lut[ty2, tx1[None, :], v].astype(np.float32)
    l22 = lut[ty2, tx2[None, :], v].astype(np.float32)
    res = (l11 * xa1 + l12 * xa) * ya1 + (l21 * xa1 + l22 * xa) * ya
    return np.clip(np.rint(res), 0, 255).astype(np.uint8)


# ---------------------------------------------------------------------------------------
# the reference's transform classes (same names, arguments and RNG draws)
# ---------------------------------------------------------------------------------------
class ElasticDeform:
    """:15-42 -- random displacement fields (uniform noise blurred by a 17x17 Gaussian,
    scaled by alpha) applied by remap: bilinear for the image, nearest for the mask."""

    def __init__(self, alpha=(20, 40), sigma=(6, 10), p=0.3):
        self.alpha, self.sigma, self.p = alpha, sigma, p

    def __call__(self, img, mask):
        if random.random() > self.p:
            return img, mask
        img_np = np.array(img)
        mask_np = np.array(mask)
        h, w = img_np.shape[:2]
        alpha = random.uniform(*self.alpha)
        sigma = random.uniform(*self.sigma)
        dx = gaussian_blur(np.random.rand(h, w) * 2 - 1, 17, sigma) * alpha
        dy = gaussian_blur(np.random.rand(h, w) * 2 - 1, 17, sigma) * alpha
        x, y = np.meshgrid(np.arange(w), np.arange(h))
        map_x = (x + dx).astype(np.float32)
        map_y = (y + dy).astype(np.float32)
        if img_np.ndim == 2:
            img_def = remap_linear_u8(img_np, map_x, map_y)
        else:
            img_def = np.stack([remap_linear_u8(img_np[..., c], map_x, map_y)
                                for c in range(img_np.shape[2])], axis=-1)
        mask_def = remap_nearest(mask_np, map_x, map_y)
        return Image.fromarray(img_def), Image.fromarray(mask_def)


class SpeckleNoise:
    """:45-54 -- multiplicative Gaussian noise on the image."""

    def __init__(self, sigma=(0.05, 0.15), p=0.5):
        self.sigma, self.p = sigma, p

    def __call__(self, img, mask):
        if random.random() > self.p:
            return img, mask
        img_np = np.array(img).astype(np.float32) / 255.
        noise = np.random.normal(0, random.uniform(*self.sigma), img_np.shape)
        img_np = img_np + img_np * noise
        img_np = np.clip(img_np * 255., 0, 255).astype(np.uint8)
        return Image.fromarray(img_np), mask


class TGCAugment:
    """:57-70 -- a random gain per horizontal depth band (time-gain compensation)."""

    def __init__(self, num_bins=10, gain=(0.8, 1.2), p=0.5):
        self.num_bins, self.gain, self.p = num_bins, gain, p

    def __call__(self, img, mask):
        if random.random() > self.p:
            return img, mask
        img_np = np.array(img).astype(np.float32)
        h = img_np.shape[0]
        bin_h = h // self.num_bins
        for i in range(self.num_bins):
            g = random.uniform(*self.gain)
            img_np[i * bin_h:(i + 1) * bin_h] *= g
        img_np = np.clip(img_np, 0, 255).astype(np.uint8)
        return Image.fromarray(img_np), mask


class CLAHE:
    """:73-81 -- contrast-limited adaptive histogram equalisation of the image."""

    def __init__(self, clip=2.0, grid=(4, 4), p=0.3):
        self.clip, self.grid, self.p = clip, grid, p

    def __call__(self, img, mask):
        if random.random() > self.p:
            return img, mask
        return Image.fromarray(clahe_u8(np.array(img), self.clip, self.grid)), mask


class AdjustBrightness:
    """:84-93 -- brightness factor U(0.5, 1.5) with probability adjust_prob."""

    def __init__(self, adjust_prob):
        self.adjust_prob = adjust_prob

    def __call__(self, image, mask):
        if random.random() < self.adjust_prob:
            factor = random.uniform(0.5, 1.5)
            image = ImageEnhance.Brightness(image).enhance(factor)
        return image, mask


class RandomCrop:
    """:95-112 -- the same crop window of image and mask."""

    def __init__(self, crop_prob, crop_width, crop_height):
        self.crop_prob = crop_prob
        self.crop_width = crop_width
        self.crop_height = crop_height

    def __call__(self, image, mask):
        if random.random() < self.crop_prob:
            width, height = image.size
            top = random.randint(0, height - self.crop_height)
            left = random.randint(0, width - self.crop_width)
            box = (left, top, left + self.crop_width, top + self.crop_height)
            image, mask = image.crop(box), mask.crop(box)
        return image, mask


class Flip:
    """:114-130 -- horizontal, then vertical, each with probability flip_prob."""

    def __init__(self, flip_prob):
        self.flip_prob = flip_prob

    def __call__(self, image, mask):
        if random.random() < self.flip_prob:
            image = image.transpose(Image.FLIP_LEFT_RIGHT)
            mask = mask.transpose(Image.FLIP_LEFT_RIGHT)
        if random.random() < self.flip_prob:
            image = image.transpose(Image.FLIP_TOP_BOTTOM)
            mask = mask.transpose(Image.FLIP_TOP_BOTTOM)
        return image, mask


class Rotate:
    """:132-141 -- rotation by U(-180, 180) degrees about the centre, nearest, same size,
    corners filled with 0."""

    def __init__(self, rotate_prob):
        self.rotate_prob = rotate_prob

    def __call__(self, image, mask):
        if random.random() < self.rotate_prob:
            angle = random.uniform(-180, 180)
            image = image.rotate(angle, Image.NEAREST, expand=False, fillcolor=0)
            mask = mask.rotate(angle, Image.NEAREST, expand=False, fillcolor=0)
        return image, mask


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


def build_train_transform(cfg, size=(512, 512), tail=None):
    """main.py:66-91: the optional ultrasound augmentations (cfg.use_elastic / use_speckle /
    use_tgc / use_clahe) around the always-on Flip(0.5), Rotate(0.5), AdjustBrightness(0.5),
    then Resize + ToTensor -- or ``tail`` (e.g. [DecodeU8()]) when the resize runs on the
    device."""
    tfs = []
    if getattr(cfg, "use_elastic", False):
        tfs.append(ElasticDeform(p=0.25))
    tfs += [Flip(0.5), Rotate(0.5), AdjustBrightness(0.5)]
    if getattr(cfg, "use_speckle", False):
        tfs.append(SpeckleNoise(p=0.3))
    if getattr(cfg, "use_tgc", False):
        tfs.append(TGCAugment(p=0.25))
    if getattr(cfg, "use_clahe", False):
        tfs.append(CLAHE(p=0.3))
    tfs += tail if tail is not None else [Resize(size), ToTensor()]
    return Compose(tfs)
