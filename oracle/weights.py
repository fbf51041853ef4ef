"""Counter-hash generator for parameters and synthetic inputs (test infra only).

The reference initialises with PyTorch's default RNG (``models/model.py:6-31``,
``init_weights`` at ``utils/utils.py:253-257`` is never called).  To make the
golden fixtures reproducible on a machine that has no reference code, every
value used by a fixture comes from this documented formula instead:

    h(t, e)  = splitmix64(seed * 0x9E3779B97F4A7C15 + (t << 36) + e)
    u(t, e)  = (h >> 11) * 2**-53                      in [0, 1)

* conv / conv-transpose weight and bias of fan-in F: ``(2u - 1) / sqrt(F)``
  (the bound of torch's default kaiming_uniform(a=sqrt(5)) init);
* BatchNorm gamma: ``gamma_lo + (gamma_hi - gamma_lo) * u``;
  BatchNorm beta: ``0.1 * (2u - 1)``;
* tensor index ``t`` is the position in ``named_parameters()`` order.

Inputs: ``x = u`` (an image in [0, 1) like ToTensor, ``utils/transforms.py:152-156``)
with tensor index 1000; targets: a union of hashed discs (a nodule phantom) so
Dice is meaningful, tensor index 2000.
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed, tensor_idx, n):
    """n uniforms in [0,1) (float64) for counter (seed, tensor_idx, 0..n-1)."""
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + (np.uint64(tensor_idx) << np.uint64(36))
        e = np.arange(n, dtype=np.uint64)
        h = splitmix64(base + e)
    return (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def fan_in(shape, transposed=False):
    if len(shape) == 1:
        return None
    if transposed:  # ConvTranspose2d weight [Cin, Cout, kh, kw]: torch uses dim 1 as fan-in
        return shape[1] * shape[2] * shape[3]
    return int(np.prod(shape[1:]))


def make_params(spec, seed=42, gamma_lo=0.5, gamma_hi=1.5):
    """spec: list of (name, shape, kind) with kind in
    {'conv_w','conv_b','convT_w','convT_b','bn_w','bn_b'}; conv_b / convT_b
    carry the fan-in of their weight as 4th element.  Returns {name: float32 ndarray}."""
    out = {}
    for t, item in enumerate(spec):
        name, shape, kind = item[0], tuple(item[1]), item[2]
        n = int(np.prod(shape))
        u = uniform(seed, t, n)
        if kind == "conv_w":
            v = (2 * u - 1) / np.sqrt(fan_in(shape))
        elif kind == "convT_w":
            v = (2 * u - 1) / np.sqrt(fan_in(shape, transposed=True))
        elif kind in ("conv_b", "convT_b"):
            v = (2 * u - 1) / np.sqrt(item[3])
        elif kind == "bn_w":
            v = gamma_lo + (gamma_hi - gamma_lo) * u
        elif kind == "bn_b":
            v = 0.1 * (2 * u - 1)
        else:
            raise ValueError(kind)
        out[name] = v.astype(np.float32).reshape(shape)
    return out


def make_input(seed, B, C, H, W):
    return uniform(seed, 1000, B * C * H * W).astype(np.float32).reshape(B, C, H, W)


def make_target(seed, B, H, W, n_discs=3):
    """Binary nodule phantom: union of n_discs hashed discs per image, float32 {0,1}."""
    u = uniform(seed, 2000, B * n_discs * 3).reshape(B, n_discs, 3)
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    t = np.zeros((B, 1, H, W), np.float32)
    for b in range(B):
        m = np.zeros((H, W), bool)
        for d in range(n_discs):
            cy, cx = u[b, d, 0] * H, u[b, d, 1] * W
            r = (0.08 + 0.17 * u[b, d, 2]) * min(H, W)
            m |= (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
        t[b, 0] = m
    return t
