"""Input pipeline on the host: the resampling plan the device kernel uses equals Pillow's
(the library's unet_resize_plan vs the restatement in oracle/resize_ref.py), and the
restatement reproduces Pillow's Image.resize(BILINEAR) bit-exactly."""
import numpy as np
import pytest

from oracle import resize_ref as RR

SIZES = [(580, 360, 512), (360, 580, 512), (256, 256, 256), (100, 37, 64), (64, 64, 512),
         (1000, 999, 256), (512, 768, 512)]


@pytest.mark.parametrize("h,w,s", SIZES)
def test_restatement_matches_pillow(h, w, s):
    from PIL import Image
    rng = np.random.default_rng(h * 7 + w)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(img, "L").resize((s, s), Image.BILINEAR))
    np.testing.assert_array_equal(RR.resize_u8(img, s, s), ref)


@pytest.mark.parametrize("n_in,n_out", [(580, 512), (360, 512), (1000, 256), (37, 64), (512, 512)])
def test_library_plan_matches_restatement(n_in, n_out):
    from unet_hip.data import resize_plan
    k, b = resize_plan(n_in, n_out)
    rk, rb = RR.plan(n_in, n_out)
    np.testing.assert_array_equal(k, rk)
    np.testing.assert_array_equal(b, rb)
