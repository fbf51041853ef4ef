"""Device input pipeline (unet_resize_u8 via unet_hip.GpuResizeToTensor) vs Pillow:
Resize + ToTensor of DDTI-like uint8 images and binary masks, bit-exact
(utils/transforms.py:143-156: TF.resize of both = Pillow BILINEAR, TF.to_tensor = u8/255)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("h,w,s", [(580, 360, 512), (360, 580, 256), (256, 256, 256),
                                   (100, 37, 64), (64, 64, 512), (1000, 999, 256)])
def test_resize_to_tensor_bit_exact(h, w, s):
    from PIL import Image
    import unet_hip
    rng = np.random.default_rng(h + 13 * w)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    yy, xx = np.mgrid[0:h, 0:w]
    mask = (((yy - h / 2) ** 2 + (xx - w / 3) ** 2) < (min(h, w) / 4) ** 2).astype(np.uint8) * 255
    pipe = unet_hip.GpuResizeToTensor((s, s), device="cuda:0")
    x, t = pipe([img, img[::-1].copy()], [mask, mask])
    torch.cuda.synchronize()
    for i, (a, m) in enumerate([(img, mask), (img[::-1].copy(), mask)]):
        ra = np.asarray(Image.fromarray(a, "L").resize((s, s), Image.BILINEAR), np.float32) / 255
        rm = np.asarray(Image.fromarray(m, "L").resize((s, s), Image.BILINEAR), np.float32) / 255
        np.testing.assert_array_equal(x[i, 0].cpu().numpy(), ra)
        np.testing.assert_array_equal(t[i, 0].cpu().numpy(), rm)


def _jpeg_dataset(root, n=4):
    from PIL import Image
    rng = np.random.default_rng(0)
    for split in ("train", "val", "test"):
        os.makedirs(root / split, exist_ok=True)
        os.makedirs(root / (split + "_mask"), exist_ok=True)
        for i in range(n):
            h, w = int(rng.integers(200, 600)), int(rng.integers(200, 600))
            img = rng.integers(0, 256, (h, w), dtype=np.uint8)
            yy, xx = np.mgrid[0:h, 0:w]
            m = (((yy - h / 2) ** 2 + (xx - w / 2) ** 2) < (min(h, w) / 4) ** 2).astype(np.uint8) * 255
            Image.fromarray(img, "L").save(root / split / f"{i}.jpg")
            Image.fromarray(m, "L").save(root / (split + "_mask") / f"{i}_mask.jpg")


def test_device_loader_matches_host_transforms(tmp_path):
    """MedicalDataset + DecodeU8 + DeviceResizeLoader == MedicalDataset + Resize + ToTensor."""
    from data.data_loader import DecodeU8, DeviceResizeLoader, MedicalDataset, u8_collate
    from utils.transforms import Compose, Resize, ToTensor
    _jpeg_dataset(tmp_path)
    d, md = str(tmp_path / "train"), str(tmp_path / "train_mask")
    host = MedicalDataset(d, md, Compose([Resize((256, 256)), ToTensor()]))
    dev = DeviceResizeLoader(torch.utils.data.DataLoader(MedicalDataset(d, md, DecodeU8()),
                                                         batch_size=4, collate_fn=u8_collate),
                             (256, 256), "cuda:0")
    x, t = next(iter(dev))
    for i in range(4):
        hx, ht = host[i]
        assert torch.equal(x[i].cpu(), hx) and torch.equal(t[i].cpu(), ht), i


def test_main_cli_gpu_transforms(tmp_path, monkeypatch):
    import main
    _jpeg_dataset(tmp_path / "ddti")
    monkeypatch.chdir(tmp_path)
    args = main.get_parser(["--mode", "both", "--dataset_path", str(tmp_path / "ddti"), "--epochs",
                            "1", "--batch_size", "2", "--image_size", "64", "--num_workers", "0",
                            "--dice_ratio", "1", "--gpu_transforms"])
    main.main(args)
    assert len(os.listdir(tmp_path / "experiments")) == 1


@pytest.mark.parametrize("mode", ["P", "1"])
@pytest.mark.parametrize("h,w,s", [(580, 360, 512), (100, 37, 64), (64, 64, 64)])
def test_palette_and_bilevel_resize_bit_exact(mode, h, w, s):
    """Palette and bilevel files: Pillow's Image.resize (TF.resize) uses NEAREST for those
    modes; DecodeU8 tags the planes and the device path matches Resize + ToTensor."""
    from PIL import Image
    import unet_hip
    from data.data_loader import DecodeU8
    from utils.transforms import Resize, ToTensor
    rng = np.random.default_rng(h * 3 + w)
    a = rng.integers(0, 256, (h, w), dtype=np.uint8)
    img = Image.fromarray(a, "P") if mode == "P" else Image.fromarray(a, "L").convert("1")
    pi, pm = DecodeU8()(img, img)
    pipe = unet_hip.GpuResizeToTensor((s, s), device="cuda:0")
    x, t = pipe([pi], [pm])
    torch.cuda.synchronize()
    hx, ht = ToTensor()(*Resize((s, s))(img, img))
    assert torch.equal(x[0].cpu(), hx) and torch.equal(t[0].cpu(), ht)
