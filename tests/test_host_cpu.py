"""Host-side mirror modules (no GPU): metrics-from-counts == the reference's array metrics,
transforms, synthetic data, CLI parsing, loss-module plumbing."""
import numpy as np
import pytest
import torch


def _counts(pred, target):
    p = pred.astype(bool)
    ti = target.astype(np.uint8)
    tb = target != 0
    return [int((p & (ti == 1)).sum()), int((p & (ti == 0)).sum()), int((~p & (ti == 1)).sum()),
            int((~p & (ti == 0)).sum()), int((p & tb).sum()), int((p | tb).sum())]


@pytest.mark.parametrize("soft", [False, True])
def test_metrics_from_counts_match_array_metrics(soft):
    from utils.utils import (calculate_acc, calculate_iou, calculate_precision_recall_f1,
                             metrics_from_counts)
    rng = np.random.default_rng(0)
    pred = (rng.random((4, 1, 32, 32)) > 0.5).astype(np.uint8)
    target = (rng.random((4, 1, 32, 32)) > 0.6).astype(np.float32)
    if soft:  # mixup soft labels (utils/trainer.py:77-78)
        target = 0.3 * target + 0.7 * (rng.random(target.shape) > 0.5)
    acc, p, r, f1, iou = metrics_from_counts(_counts(pred, target))
    assert acc == pytest.approx(calculate_acc(pred, target))
    pp, rr, ff = calculate_precision_recall_f1(pred, target)
    assert (p, r, f1) == pytest.approx((pp, rr, ff))
    assert iou == pytest.approx(calculate_iou(pred, target))


def test_global_metrics():
    from utils.utils import global_metrics_from_counts
    m = global_metrics_from_counts([10, 5, 3, 82])
    assert m["IoU"] == pytest.approx(10 / 18, rel=1e-6)
    assert m["F1"] == pytest.approx(2 * (10 / 15) * (10 / 13) / (10 / 15 + 10 / 13), rel=1e-6)


def test_transforms_and_synthetic():
    from PIL import Image
    from data.data_loader import SyntheticSegmentation
    from utils.transforms import Compose, Resize, ToTensor
    img = Image.fromarray((np.arange(40 * 30) % 256).astype(np.uint8).reshape(40, 30))
    mask = Image.fromarray(((np.arange(40 * 30) % 7) == 0).astype(np.uint8).reshape(40, 30) * 255)
    a, m = Compose([Resize((64, 48)), ToTensor()])(img, mask)
    assert a.shape == (1, 64, 48) and m.shape == (1, 64, 48)
    assert 0 <= a.min() and a.max() <= 1 and 0 <= m.min() and m.max() <= 1
    # TF.resize (utils/transforms.py:147-148) resizes the mask BILINEARLY too: soft targets
    ref = np.asarray(mask.resize((48, 64), Image.BILINEAR), np.float32) / 255
    assert np.array_equal(m[0].numpy(), ref) and len(torch.unique(m)) > 2
    ds = SyntheticSegmentation(3, 64)
    x, y = ds[1]
    assert x.shape == (1, 64, 64) and y.shape == (1, 64, 64) and y.sum() > 0
    assert torch.equal(ds[1][0], x)


def test_cli_flags_match_reference():
    import main
    a = main.get_parser([])
    for k, v in dict(bce_ratio=1, dice_ratio=0, focal_ratio=1, boundary_ratio=0, lr=1e-5,
                     batch_size=16, epochs=10000, mixup_alpha=0.2, mixup_prob=0.3,
                     early_stop_patience=50, use_data_parallel=True, use_amp_autocast=False).items():
        assert getattr(a, k) == v, k


def test_boundary_loss_matches_reference_formula():
    import scipy.ndimage as nd
    from models.loss import BoundaryLoss
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.standard_normal((2, 1, 16, 16)).astype(np.float32))
    t = torch.from_numpy((rng.random((2, 1, 16, 16)) > 0.7).astype(np.float32))
    ref = 0.0
    for b in range(2):
        d = torch.from_numpy(nd.distance_transform_edt(1 - t[b, 0].numpy().astype(np.uint8))).float()
        ref += torch.mean(torch.abs(torch.sigmoid(x[b, 0]) - t[b, 0]) * d)
    assert float(BoundaryLoss()(x, t)) == pytest.approx(float(ref / 2), rel=1e-6)


def test_to_tensor_keeps_the_image_mode():
    """utils/transforms.py ToTensor = TF.to_tensor per image: bands kept, u8 / 255."""
    from PIL import Image
    from data.data_loader import DecodeU8
    from utils.transforms import ToTensor
    rng = np.random.default_rng(4)
    rgb = rng.integers(0, 256, (20, 30, 3), dtype=np.uint8)
    gray = rng.integers(0, 256, (20, 30), dtype=np.uint8)
    a, m = ToTensor()(Image.fromarray(rgb, "RGB"), Image.fromarray(gray, "L"))
    assert a.shape == (3, 20, 30) and m.shape == (1, 20, 30)
    assert torch.equal(a, torch.from_numpy(rgb).permute(2, 0, 1).float().div(255))
    assert torch.equal(m[0], torch.from_numpy(gray).float().div(255))
    bil = Image.fromarray(gray > 128).convert("1")
    _, b = ToTensor()(bil, bil)
    assert torch.equal(b[0], torch.from_numpy((gray > 128).astype(np.float32)))
    u8 = DecodeU8()
    assert np.array_equal(u8(bil, Image.fromarray(gray, "L"))[0], (gray > 128).astype(np.uint8) * 255)
    with pytest.raises(ValueError):
        u8(Image.fromarray(rgb, "RGB"), Image.fromarray(gray, "L"))


def test_hip_adamw_rebuilds_flat_moments_from_loaded_state():
    """HipAdamW keeps self.state as the source of truth: after load_state_dict the flat
    moment arenas are rebuilt from the loaded exp_avg / exp_avg_sq (host-side logic; the
    device update itself is covered by the GPU tests)."""
    import unet_hip
    flat = torch.arange(10, dtype=torch.float32)
    ps = [torch.nn.Parameter(flat[0:4].view(2, 2)), torch.nn.Parameter(flat[4:10])]
    opt = unet_hip.HipAdamW(ps, lr=1e-3)
    sd = {"state": {0: {"step": torch.tensor(3.0), "exp_avg": torch.full((2, 2), 0.5),
                        "exp_avg_sq": torch.full((2, 2), 0.25)},
                    1: {"step": torch.tensor(3.0), "exp_avg": torch.arange(6.0),
                        "exp_avg_sq": torch.arange(6.0) * 2}},
          "param_groups": opt.state_dict()["param_groups"]}
    opt.load_state_dict(sd)
    m, v = opt._rebuild_flat(ps, flat)
    assert torch.equal(m, torch.cat([torch.full((4,), 0.5), torch.arange(6.0)]))
    assert torch.equal(v, torch.cat([torch.full((4,), 0.25), torch.arange(6.0) * 2]))
    assert opt._views_of(ps, m, v)
    assert opt.state[ps[1]]["exp_avg"].data_ptr() == m.data_ptr() + 4 * 4
    opt.load_state_dict(sd)  # fresh tensors again: no longer views of the arenas
    assert not opt._views_of(ps, m, v)
