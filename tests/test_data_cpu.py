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


@pytest.mark.parametrize("n,bs,world", [(10, 4, 2), (37, 8, 3), (5, 4, 4), (16, 16, 8), (3, 2, 4),
                                         (2 * 256 + 3, 256, 8), (256 + 5, 256, 4)])
@pytest.mark.parametrize("shuffle", [False, True])
def test_dataparallel_shard_sampler(n, bs, world, shuffle):
    """Every rank's shards concatenate to the reference loader's global batch
    (data/data_loader.py:29-33, drop_last=False) split with torch.chunk exactly as
    nn.DataParallel scatters it (utils/trainer.py:28-30); every sample once per epoch."""
    import torch
    from data.data_loader import DataParallelShardSampler
    samplers = [DataParallelShardSampler(n, bs, shuffle, r, world, seed=3) for r in range(world)]
    for ep in (0, 1):
        for s in samplers:
            s.set_epoch(ep)
        per_rank = [list(s) for s in samplers]
        assert all(len(p) == len(samplers[0]) == (n + bs - 1) // bs for p in per_rank)
        seen = []
        for b, glob in enumerate(samplers[0].global_batches()):
            chunks = torch.chunk(glob, world)
            for r in range(world):
                want = chunks[r].tolist() if r < len(chunks) else []
                assert per_rank[r][b] == want
            seen += glob.tolist()
        assert sorted(seen) == list(range(n))


@pytest.mark.parametrize("h,w,oh,ow", [(580, 360, 512, 512), (37, 100, 64, 64), (2999, 17, 256, 1000),
                                       (64, 64, 64, 64), (7, 3, 513, 1)])
def test_nearest_restatement_matches_pillow(h, w, oh, ow):
    """Pillow resizes palette ("P") and bilevel ("1") images with NEAREST whatever filter
    TF.resize asks for (Image.resize); the restatement and the library's one-tap plan
    reproduce it."""
    from PIL import Image
    from unet_hip.data import nearest_plan
    rng = np.random.default_rng(h * 31 + w)
    idx = rng.integers(0, 256, (h, w), dtype=np.uint8)
    pal = Image.fromarray(idx, "P")
    ref = np.asarray(pal.resize((ow, oh), Image.BILINEAR))
    np.testing.assert_array_equal(RR.resize_nearest_u8(idx, oh, ow), ref)
    bits = Image.fromarray((idx > 127).astype(np.uint8) * 255, "L").convert("1", dither=Image.Dither.NONE)
    rb = np.asarray(bits.resize((ow, oh), Image.BILINEAR).convert("L"))
    np.testing.assert_array_equal(RR.resize_nearest_u8(np.asarray(bits.convert("L")), oh, ow), rb)
    for n_in, n_out in ((w, ow), (h, oh)):
        k, b = nearest_plan(n_in, n_out)
        assert (k == 1 << 22).all() and (b[:, 1] == 1).all()
        np.testing.assert_array_equal(b[:, 0], RR.nearest_index(n_in, n_out))


def test_decode_u8_modes_match_to_tensor():
    """DecodeU8 planes / 255 == the host ToTensor (TF.to_tensor) for "L", "P" and "1";
    "P" / "1" planes are tagged for NEAREST and keep the tag through pickling (workers);
    multi-band images are refused."""
    import pickle
    import torch
    from PIL import Image
    from data.data_loader import DecodeU8
    from utils.transforms import ToTensor
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, (40, 30), dtype=np.uint8)
    for mode, img in (("L", Image.fromarray(a, "L")), ("P", Image.fromarray(a, "P")),
                      ("1", Image.fromarray(a, "L").convert("1"))):
        pl, _ = DecodeU8()(img, img)
        assert pl.resample == ("bilinear" if mode == "L" else "nearest")
        assert pickle.loads(pickle.dumps(pl)).resample == pl.resample
        want, _ = ToTensor()(img, img)
        got = torch.from_numpy(np.asarray(pl, np.float32) / np.float32(255.0))[None]
        assert torch.equal(got, want), mode
    with pytest.raises(ValueError):
        DecodeU8()(Image.fromarray(np.zeros((4, 4, 3), np.uint8), "RGB"), None)
