"""NumPy restatement of the exact three-way bf16 split (csrc/x3_split.h) the x3 GEMMs stream
(test infrastructure: tests/test_lib_cpu.py checks the library's host hook against it, and
tests/test_gpu_x3.py the device pass).

  normal v:             h = rne(v), m = rne(v - h), l = rne(v - h - m)   (h + m + l == v)
  |v| >= 0x1.FFp127:    h = the largest finite bf16 of v's sign (rne would overflow)
  +-inf, NaN:           h = v, m = l = 0
  subnormal pieces:     bf16 has f32's exponent range but a 2^-133 subnormal quantum
"""
import numpy as np

BF16_OVF = np.float32(np.ldexp(0x1FF, 127 - 8))   # 0x1.FFp127: rounds to inf in bf16
BF16_MAX = np.float32(np.ldexp(0x1FE, 127 - 8))   # 0x1.FEp127: largest finite bf16
F32_MAX = np.float32(np.finfo(np.float32).max)


def rne_bits(v):
    """float32 -> bf16 bit patterns, round to nearest even; NaN -> quiet NaN."""
    u = np.asarray(v, np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    r = np.where(nan, (u >> 16) | 0x40, r)
    return r.astype(np.uint16)


def bf16_to_f32(b):
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


def split(v):
    """(h, m, l) bf16 bit patterns of float32 array v."""
    v = np.asarray(v, np.float32)
    a = np.abs(v)
    with np.errstate(invalid="ignore", over="ignore"):
        huge = (a >= BF16_OVF) & (a <= F32_MAX)
        h = rne_bits(np.where(huge, np.copysign(BF16_MAX, v), v).astype(np.float32))
        r1 = (v - bf16_to_f32(h)).astype(np.float32)
        r1 = np.where(a <= F32_MAX, r1, np.float32(0)).astype(np.float32)
        m = rne_bits(r1)
        lo = rne_bits((r1 - bf16_to_f32(m)).astype(np.float32))
    return h, m, lo


def to_image(h, m, lo):
    """[n / 32][3][32] x3 image layout (include/unet_hip.h unet_x3_split_*)."""
    n = h.size
    img = np.empty((n // 32, 3, 32), np.uint16)
    img[:, 0] = h.reshape(-1, 32)
    img[:, 1] = m.reshape(-1, 32)
    img[:, 2] = lo.reshape(-1, 32)
    return img.reshape(-1)


def from_image(img):
    img = np.asarray(img, np.uint16).reshape(-1, 3, 32)
    return img[:, 0].reshape(-1), img[:, 1].reshape(-1), img[:, 2].reshape(-1)


def edge_values(seed=0):
    """Normal values over the whole exponent range plus the range edges, padded to a multiple
    of 32: huge finite (around the bf16 overflow threshold and FLT_MAX), +-inf, NaN,
    subnormal and tiny normal values, signed zeros."""
    rng = np.random.default_rng(seed)
    normal = (rng.uniform(1, 2, 2048) * np.exp2(rng.integers(-126, 127, 2048))
              * rng.choice([-1, 1], 2048)).astype(np.float32)
    below = np.nextafter(BF16_OVF, np.float32(0))
    huge = np.array([BF16_MAX, below, BF16_OVF, np.nextafter(BF16_OVF, np.float32(np.inf)),
                     np.float32(3.395e38), F32_MAX], np.float32)
    huge = np.concatenate([huge, -huge])
    special = np.array([np.inf, -np.inf, np.nan, 0.0, -0.0], np.float32)
    tiny = np.array([1e-45, -1e-45, 1e-40, -3.3e-39, 1.1754942e-38, 1.1754944e-38,
                     np.ldexp(1.2345, -110), -np.ldexp(1.75, -120), np.ldexp(1.999, -127)],
                    np.float32)
    v = np.concatenate([normal, huge, special, tiny]).astype(np.float32)
    pad = (-v.size) % 32
    return np.concatenate([v, rng.uniform(-1, 1, pad).astype(np.float32)])
