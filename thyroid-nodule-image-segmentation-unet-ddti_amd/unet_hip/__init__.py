"""unet_hip - MI355X-native (gfx950) UNet training / inference path for the DDTI
thyroid-nodule workload (drop-in for models/model.py:UNet of
WuJiaqiii/Thyroid-nodule-image-segmentation-UNet-DDTI).

    from unet_hip import UNet, seg_losses, HipAdamW

Everything on the hot path runs in libunet_hip.so (hand-written HIP kernels, C ABI in
include/unet_hip.h); this package is the PyTorch-facing host side.  There is no CPU
fallback: without the built library every entry point raises ``HipUnavailable``.
"""
from ._lib import HipError, HipUnavailable, LIB_PATH, load  # noqa: F401
from .data import GpuResizeToTensor  # noqa: F401
from .functional import seg_losses  # noqa: F401
from .module import ModUNet, ResUNet, UNet  # noqa: F401
from .optim import HipAdamW  # noqa: F401
from .runtime import UNetRuntime  # noqa: F401
