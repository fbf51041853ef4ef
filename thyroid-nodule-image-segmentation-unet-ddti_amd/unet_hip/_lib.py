"""ctypes binding of libunet_hip.so (include/unet_hip.h).

The library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()``) into
``lib/libunet_hip.so``.  There is deliberately no fallback: if the library is missing or
does not load, every entry point raises ``HipUnavailable`` -- the product path never
silently runs on CPU/PyTorch kernels.

``torch`` is imported before the library is opened so that the process has exactly one
HIP runtime (torch's ``libamdhip64.so.7``; the library's NEEDED entry resolves to it by
soname), which makes torch tensors' device pointers and streams valid in the library.
"""
import ctypes
import os

import torch  # noqa: F401  (must be loaded first: shared HIP runtime)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("UNET_HIP_LIB", os.path.join(PKG_DIR, "lib", "libunet_hip.so"))
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "unet_hip.h")


class HipUnavailable(RuntimeError):
    pass


class HipError(RuntimeError):
    pass


STATUS = {0: "UNET_OK", -1: "UNET_ERR_INVALID", -2: "UNET_ERR_SHAPE", -3: "UNET_ERR_HIP",
          -4: "UNET_ERR_WORKSPACE", -5: "UNET_ERR_UNSUPPORTED", -6: "UNET_ERR_NOMEM",
          -7: "UNET_ERR_INTERNAL"}

c_int, c_int64, c_float, c_double, c_size_t = (ctypes.c_int, ctypes.c_int64, ctypes.c_float,
                                                ctypes.c_double, ctypes.c_size_t)
c_void_p, c_char_p = ctypes.c_void_p, ctypes.c_char_p
P = ctypes.POINTER


class UnetCfg(ctypes.Structure):
    _fields_ = [("in_channels", c_int), ("out_channels", c_int), ("variant", c_int),
                ("base_filters", c_int), ("depth", c_int), ("math", c_int)]


VARIANT_MODEL = 0  # models/model.py:UNet
VARIANT_MOD = 1    # models/mod.py:UNet
VARIANT_RES = 2    # models/mod.py:ResUNet
MATH_F32 = 0       # conv GEMMs on f32 MFMA (exact f32 products)
MATH_BF16 = 1      # conv GEMMs on bf16 MFMA, f32 accumulate (BASELINE config 4)


# name -> (restype, argtypes); mirrors include/unet_hip.h
SIGNATURES = {
    "unet_create": (c_int, [P(UnetCfg), c_int, P(c_void_p)]),
    "unet_destroy": (c_int, [c_void_p]),
    "unet_last_error": (c_char_p, [c_void_p]),
    "unet_num_params": (c_int, [c_void_p, P(c_int), P(c_int64)]),
    "unet_param_info": (c_int, [c_void_p, c_int, P(c_char_p), P(c_int), P(c_int64), P(c_int64)]),
    "unet_num_bn": (c_int, [c_void_p, P(c_int), P(c_int64)]),
    "unet_bn_info": (c_int, [c_void_p, c_int, P(c_char_p), P(c_int), P(c_int64)]),
    "unet_workspace_size": (c_int, [c_void_p, c_int, c_int, c_int, c_int, P(c_size_t)]),
    "unet_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_size_t, c_int, c_int, c_int, c_int, c_void_p]),
    "unet_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int,
                              c_int, c_int, c_void_p]),
    "unet_loss_stats": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                c_void_p, c_void_p, c_void_p]),
    "unet_loss_finalize": (c_int, [c_void_p, c_void_p, c_void_p, c_float, c_float, c_float,
                                   c_void_p]),
    "unet_loss_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                              c_void_p, c_void_p, c_float, c_float, c_float, c_void_p]),
    "unet_loss_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_float, c_float, c_float, c_void_p]),
    "unet_adamw": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int,
                           c_double, c_double, c_double, c_double, c_double, c_double, c_void_p]),
    "unet_adamw_repack": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int,
                                  c_double, c_double, c_double, c_double, c_double, c_double, c_void_p]),
    "unet_params_changed": (c_int, [c_void_p]),
    "unet_set_option": (c_int, [c_void_p, c_char_p, c_int64]),
    "unet_get_option": (c_int, [c_void_p, c_char_p, P(c_int64)]),
    "unet_mask_counts": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                 c_void_p]),
    "unet_num_buckets": (c_int, [c_void_p, P(c_int)]),
    "unet_bucket_range": (c_int, [c_void_p, c_int, P(c_int64), P(c_int64)]),
    "unet_stream_wait_bucket": (c_int, [c_void_p, c_int, c_void_p]),
    "unet_bucket_event": (c_int, [c_void_p, c_int, P(c_void_p)]),
    "unet_option_name": (c_int, [c_int, P(c_char_p)]),
    "unet_debug_view": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, P(c_int64),
                                P(c_int64), P(c_int), P(c_int)]),
    "unet_resize_plan": (c_int, [c_int, c_int, c_void_p, c_void_p, P(c_int)]),
    "unet_resize_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                               c_void_p, c_int, c_void_p, c_void_p, c_int, c_float, c_void_p]),
    "unet_x3_split_host": (c_int, [c_void_p, c_int64, c_void_p]),
    "unet_x3_split_device": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "unet_timing_enable": (c_int, [c_void_p, c_int]),
    "unet_timing_filter": (c_int, [c_void_p, c_char_p]),
    "unet_timing_reset": (c_int, [c_void_p]),
    "unet_timing_count": (c_int, [c_void_p, P(c_int)]),
    "unet_timing_read": (c_int, [c_void_p, c_int, P(c_char_p), P(c_int64), P(c_double),
                                 P(c_double)]),
}

_lib = None
_load_error = None


def load():
    """Open libunet_hip.so once; raise HipUnavailable (never fall back) if it cannot load."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise HipUnavailable(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"{LIB_PATH} not built; run __graft_entry__.build() "
                       f"(make -C csrc) -- there is no CPU fallback")
        raise HipUnavailable(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        _load_error = f"cannot load {LIB_PATH}: {e}"
        raise HipUnavailable(_load_error) from e
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def option_names():
    """Every kernel-schedule option name the library accepts (unet_option_name)."""
    lib = load()
    out, i = [], 0
    while True:
        n = c_char_p()
        if lib.unet_option_name(i, ctypes.byref(n)) != 0:
            return out
        out.append(n.value.decode())
        i += 1


def check(rc, ctx=None, what=""):
    if rc != 0:
        msg = ""
        if ctx:
            m = load().unet_last_error(ctx)
            msg = m.decode() if m else ""
        raise HipError(f"{what}: {STATUS.get(rc, rc)} {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
