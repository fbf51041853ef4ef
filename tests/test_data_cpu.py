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


@pytest.mark.parametrize("n,bs,world", [(10, 4, 2), (37, 8, 3), (5, 4, 4), (16, 16, 8), (3, 2, 4)])
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
