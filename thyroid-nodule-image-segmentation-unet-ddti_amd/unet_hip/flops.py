"""Algorithmic work of one training step: the per-unit figure behind
``bench.py``'s roofline.

Counted: every conv / ConvTranspose / 1x1 head multiply-accumulate x 2 FLOP, for the
forward, the input gradient (dgrad) and the weight gradient (wgrad); the first conv has
no input gradient.  BN, ReLU, pooling, losses and AdamW are not counted (bandwidth work).

    models/model.py UNet, 256x256:       288,475,840,512 FLOP / image
    models/mod.py UNet(128, 5), 512x512: 5,709,420,822,528 FLOP / image
    models/mod.py ResUNet(64, 5), 512x512 (what the reference main.py:122 trains):
        res_train_flops_per_image -- the same 3x3 / ConvT work plus every block's 1x1 skip

(The oracle's own counters, oracle/*_ref_cpu.py, are pinned to the same numbers by
tests/test_host_cpu.py.)
"""


def unet_level_macs(H, W, in_channels, out_channels, base, depth):
    """Forward MACs of the encoder/bottleneck/decoder topology shared by models/model.py
    (base 64, depth 4) and models/mod.py (any base / depth): two 3x3 convs per block,
    ConvT 2x2 s2 into every decoder level, 1x1 head."""
    macs = 0
    prev = in_channels
    for i in range(depth + 1):                    # encoders + bottleneck
        c = base << i
        hw = (H >> i) * (W >> i)
        macs += hw * 9 * (prev * c + c * c)
        prev = c
    for lv in range(depth - 1, -1, -1):           # ConvT into level lv, then its block
        c = base << lv
        hw_in = (H >> (lv + 1)) * (W >> (lv + 1))
        macs += hw_in * (2 * c) * c * 4
        hw = (H >> lv) * (W >> lv)
        macs += hw * 9 * (2 * c * c + c * c)
    macs += H * W * base * out_channels
    return macs


def train_flops_per_image(H, W, base=64, depth=4, in_channels=1, out_channels=1):
    """fwd + dgrad + wgrad = 6 x forward MACs, minus the first conv's unneeded dgrad."""
    macs = unet_level_macs(H, W, in_channels, out_channels, base, depth)
    return 6 * macs - 2 * (H * W * 9 * base * in_channels)


def res_skip_macs(H, W, in_channels, base, depth):
    """Forward MACs of ResUNet's 1x1 skip convs (models/mod.py:83): one per block, Cin ->
    Cout at the block's resolution (the decoders' Cin is the 2c-channel concat)."""
    macs = 0
    prev = in_channels
    for i in range(depth + 1):
        c = base << i
        macs += (H >> i) * (W >> i) * prev * c
        prev = c
    for lv in range(depth - 1, -1, -1):
        c = base << lv
        macs += (H >> lv) * (W >> lv) * 2 * c * c
    return macs


def res_train_flops_per_image(H, W, base=64, depth=5, in_channels=1, out_channels=1):
    """ResUNet: fwd + dgrad + wgrad of the UNet topology plus the skips, minus the first
    block's unneeded input gradients (its 3x3 conv and its skip)."""
    macs = unet_level_macs(H, W, in_channels, out_channels, base, depth) + \
        res_skip_macs(H, W, in_channels, base, depth)
    return 6 * macs - 2 * (H * W * 9 * base * in_channels) - 2 * (H * W * base * in_channels)
