"""Drop-ins for ``UNet`` (:9-66) and ``ResUNet`` (:71-131) of the reference's ``models/mod.py``.

``from models.mod import UNet`` gives the MI355X-native version of that network: the
same constructor ``UNet(in_channels=1, out_channels=1, base_filters=64, depth=5,
**kwargs)``, the same submodule tree and parameter / buffer names (encoders.*, pools,
bottleneck, upconvs.*, decoders.*, final_conv), the same block order (bias-free
Conv3x3 -> BN -> ReLU) and concat order ``[skip, up]``; forward and backward run as HIP
kernels in libunet_hip.so.  ``ResUNet`` (the network the reference's main.py:122
builds) keeps its tree too (``encoders.i.conv.*``, ``encoders.i.skip``, ...).  The other
networks of models/mod.py (ASPPUNet, ...) are outside the accelerated path
and are not provided here.
"""
from unet_hip.module import ModUNet as UNet  # noqa: F401
from unet_hip.module import ResUNet  # noqa: F401

__all__ = ["UNet", "ResUNet"]
