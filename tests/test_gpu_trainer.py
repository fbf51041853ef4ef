"""GPU: the reference-shaped plugin surface (utils/trainer.Trainer, main.py, checkpoints)
drives the HIP path end to end."""
import argparse
import os

import numpy as np
import pytest
import torch

from oracle import unet_ref_cpu as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _config(tmp, **kw):
    from utils.utils import Config
    ns = argparse.Namespace(model_type="UNet", lr=1e-4, bce_ratio=1.0, dice_ratio=1.0,
                            focal_ratio=0.5, boundary_ratio=0.0, use_mixup=True, mixup_prob=0.5,
                            mixup_alpha=0.2, epochs=2, early_stop_patience=5, batch_size=2,
                            num_workers=0)
    for k, v in kw.items():
        setattr(ns, k, v)
    cfg = Config(ns, base_dir=str(tmp))
    cfg.device = DEV
    return cfg


def test_trainer_epoch_validate_test_and_checkpoints(tmp_path):
    from data.data_loader import SyntheticSegmentation, create_dataloader
    from models.model import UNet
    from utils.trainer import Trainer
    from utils.utils import create_logger, metrics_from_counts
    cfg = _config(tmp_path, boundary_ratio=0.1)
    loaders = tuple(create_dataloader(SyntheticSegmentation(4, 64, seed=s), cfg, shuffle=(s == 0))
                    for s in range(3))
    torch.manual_seed(0)
    model = UNet()
    tr = Trainer(cfg, loaders, create_logger(os.path.join(cfg.log_dir, "t.log")), model)
    loss0 = tr.train_one_epoch(0)
    vloss, viou = tr.validate(0)
    assert np.isfinite(loss0) and np.isfinite(vloss) and 0 <= viou <= 1
    tr.train()
    best = os.path.join(cfg.model_dir, "UNet_best.pth")
    last = os.path.join(cfg.model_dir, "UNet_last.pth")
    assert os.path.exists(best) and os.path.exists(last)
    sd = torch.load(last, weights_only=True)
    assert [k for k in sd if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))] \
        == [s[0] for s in O.param_spec()]
    # the checkpoint loads into a fresh module and reproduces the eval logits
    m2 = UNet()
    m2.load_state_dict(sd)
    m2 = m2.to(DEV).eval()
    tr.model.eval()
    x = loaders[2].dataset[0][0][None].to(DEV)
    with torch.no_grad():
        assert torch.equal(m2(x), tr.model(x))
    # device-side test metrics == host metrics over the same predictions
    m = tr.test()
    preds, gts = [], []
    with torch.no_grad():
        for xb, yb in loaders[2]:
            preds.append((torch.sigmoid(tr.model(xb.to(DEV))) > 0.5).cpu().numpy().astype(np.uint8))
            gts.append(yb.numpy().astype(np.uint8))
    p, g = np.concatenate(preds).ravel(), np.concatenate(gts).ravel()
    assert m["TP"] == int(((p == 1) & (g == 1)).sum()) and m["TN"] == int(((p == 0) & (g == 0)).sum())


def test_trainer_step_matches_oracle(tmp_path):
    """One Trainer step with ratios bce=1, dice=1 == the oracle step (loss and updated params)."""
    from models.model import UNet
    from utils.trainer import Trainer
    from utils.utils import create_logger
    from _helpers import inputs
    x, t = inputs(1, 2, 64, 64)
    cfg = _config(tmp_path, use_mixup=False, focal_ratio=0.0, lr=1e-5)
    P = O.make_params(42)
    model = UNet()
    model.load_state_dict({**P, **O.init_buffers()})
    tr = Trainer(cfg, ([(x, t)], [(x, t)], [(x, t)]), create_logger(os.path.join(cfg.log_dir, "s.log")),
                 model)
    loss = tr.train_one_epoch(0)
    ref = O.train_step(P, O.init_buffers(), O.AdamWState(P, lr=1e-5), x, t)
    assert abs(loss - ref["loss"].item()) < 1e-5
    got = dict(tr.model.named_parameters())
    worst = max(float((got[k].detach().cpu() - v).abs().max()) for k, v in P.items())
    assert worst <= 4e-5  # <= 2 lr for sign-noise elements (see test_gpu_parity), 1e-7 elsewhere


def test_main_cli_synthetic(tmp_path, monkeypatch):
    import main
    monkeypatch.chdir(tmp_path)
    args = main.get_parser(["--mode", "both", "--synthetic", "4", "--epochs", "1", "--batch_size", "2",
                            "--image_size", "64", "--num_workers", "0", "--dice_ratio", "1"])
    main.main(args)
    runs = os.listdir(tmp_path / "experiments")
    assert len(runs) == 1
    assert os.path.exists(tmp_path / "experiments" / runs[0] / "models" / "UNet_last.pth")


def test_main_cli_resunet(tmp_path, monkeypatch):
    """The network the reference's main.py:122 builds (mod.py:ResUNet), through main.py."""
    import main
    monkeypatch.chdir(tmp_path)
    args = main.get_parser(["--mode", "both", "--synthetic", "4", "--epochs", "1", "--batch_size", "2",
                            "--image_size", "64", "--num_workers", "0", "--dice_ratio", "1",
                            "--model_type", "ResUNet", "--depth", "3"])
    main.main(args)
    runs = os.listdir(tmp_path / "experiments")
    assert len(runs) == 1
    assert os.path.exists(tmp_path / "experiments" / runs[0] / "models" / "ResUNet_last.pth")
