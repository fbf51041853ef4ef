"""Drop-in for the reference's ``models/model.py``.

``from models.model import UNet`` gives the MI355X-native UNet: same constructor
signature ``UNet(in_channels=1, out_channels=1)`` (reference models/model.py:6), same
``forward(x) -> logits`` contract (:53-73), same parameter / buffer names, shapes and
torch layouts (state_dicts load in both directions), but forward and backward run as
hand-written HIP kernels in libunet_hip.so.  See unet_hip/module.py.
"""
from unet_hip.module import UNet  # noqa: F401

__all__ = ["UNet"]
