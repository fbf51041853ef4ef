"""Data loading (mirror of the reference's data/data_loader.py).

``MedicalDataset(img_dir, mask_dir, transform)`` pairs ``<name>.jpg`` with
``<stem>_mask.jpg`` exactly like the reference (:9-27); ``create_dataloader`` is the same
plain DataLoader (:29-33).  ``SyntheticSegmentation`` provides device-free synthetic
batches (images in [0, 1), binary nodule-like disc masks) for benchmarks and tests, since
the DDTI data is not distributed with the code.

Device-side transforms: ``MedicalDataset(..., transform=DecodeU8())`` + ``u8_collate``
keep the host to JPEG decoding; ``DeviceResizeLoader`` then runs the reference's
Resize + ToTensor (utils/transforms.py:143-156) on the GPU (unet_hip.GpuResizeToTensor,
bit-identical to the Pillow path) and yields device batches.
"""
import os
from pathlib import Path

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset


class MedicalDataset(Dataset):
    def __init__(self, img_dir, mask_dir, transform=None):
        self.img_dir, self.mask_dir, self.transform = img_dir, mask_dir, transform
        self.img_names = [p.name for p in Path(img_dir).rglob("*")]
        self.mask_names = [n.split(".jpg")[0] + "_mask.jpg" for n in self.img_names]

    def __len__(self):
        return len(self.img_names)

    def __getitem__(self, idx):
        from PIL import Image
        img = Image.open(os.path.join(self.img_dir, self.img_names[idx]))
        mask = Image.open(os.path.join(self.mask_dir, self.mask_names[idx]))
        if self.transform:
            img, mask = self.transform(img, mask)
        return img, mask


class SyntheticSegmentation(Dataset):
    """n samples of (1, H, W) float images in [0, 1) and {0, 1} masks of 1-3 discs."""

    def __init__(self, n, size=256, seed=0):
        self.n, self.size, self.seed = n, size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        rng = np.random.default_rng(self.seed * 1_000_003 + idx)
        S = self.size
        img = rng.random((1, S, S), dtype=np.float32)
        yy, xx = np.mgrid[0:S, 0:S]
        m = np.zeros((S, S), bool)
        for _ in range(rng.integers(1, 4)):
            cy, cx = rng.random(2) * S
            r = (0.08 + 0.17 * rng.random()) * S
            m |= (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
        img[0][m] = 0.5 * img[0][m] + 0.4  # brighter nodule
        return torch.from_numpy(img), torch.from_numpy(m[None].astype(np.float32))


def create_dataloader(dataset, config, shuffle):
    return DataLoader(dataset=dataset, batch_size=config.batch_size, shuffle=shuffle,
                      num_workers=config.num_workers)


class DataParallelShardSampler(torch.utils.data.Sampler):
    """Batch sampler giving one rank of a one-process-per-GPU run exactly its
    nn.DataParallel share of the reference loader's batches.

    The reference loads GLOBAL batches of ``batch_size`` (data/data_loader.py:29-33:
    shuffle, drop_last=False, so the last batch may be short) and DataParallel scatters each
    one with torch.chunk over the replicas (utils/trainer.py:28-30).  Here every rank draws
    the same batch order (shared seed, re-drawn per epoch by ``set_epoch``) and yields its
    torch.chunk slice of every batch.  The slice is empty for a last batch with fewer
    samples than ranks; ``dp_collate`` turns that into ``None`` and the Trainer then joins
    the step's collectives with zero contributions (``DistributedUNet.empty_step``)."""

    def __init__(self, n, batch_size, shuffle, rank, world, seed=0):
        self.n, self.batch_size, self.shuffle = int(n), int(batch_size), bool(shuffle)
        self.rank, self.world, self.seed, self.epoch = int(rank), int(world), int(seed), 0

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def global_batches(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g)
        else:
            order = torch.arange(self.n)
        return [order[b:b + self.batch_size] for b in range(0, self.n, self.batch_size)]

    def __iter__(self):
        for batch in self.global_batches():
            chunks = torch.chunk(batch, self.world)
            yield chunks[self.rank].tolist() if self.rank < len(chunks) else []

    def __len__(self):
        return (self.n + self.batch_size - 1) // self.batch_size


def dp_collate(collate=None):
    """Collate for DataParallelShardSampler: an empty shard becomes None."""
    from torch.utils.data import default_collate
    inner = collate or default_collate

    def fn(batch):
        return None if len(batch) == 0 else inner(batch)
    return fn


class U8Plane(np.ndarray):
    """A decoded (H, W) uint8 plane that remembers which filter Pillow's resize would use
    for its source image: ``"nearest"`` for palette ("P") and bilevel ("1") images, for
    which Image.resize replaces BILINEAR by NEAREST, else ``"bilinear"``."""

    resample = "bilinear"

    def __array_finalize__(self, obj):
        self.resample = getattr(obj, "resample", "bilinear")

    def __reduce__(self):  # DataLoader workers pickle samples: keep the tag
        fn, args, state = super().__reduce__()
        return fn, args, (state, self.resample)

    def __setstate__(self, st):
        state, self.resample = st
        super().__setstate__(state)

    @staticmethod
    def of(a, resample):
        p = np.ascontiguousarray(a, dtype=np.uint8).view(U8Plane)
        p.resample = resample
        return p


class DecodeU8:
    """Transform that only decodes: (PIL image, PIL mask) -> two (H, W) uint8 planes.

    The device pipeline is single-band 8-bit, as TF.to_tensor sees it: "L" gives the
    pixel values; "P" (palette) the raw palette indices (to_tensor divides the indices by
    255); "1" 0 / 255 (to_tensor's {0, 1} after its x255 and /255).  For "P" and "1" the
    planes are tagged ``resample="nearest"``: Pillow's Image.resize (which TF.resize calls)
    resizes those modes with NEAREST whatever filter is asked for.  Multi-band or
    non-8-bit modes (RGB, I;16, F, ...) would give a different tensor there and are
    refused rather than silently converted."""

    @staticmethod
    def _plane(pic):
        if pic.mode == "L":
            return U8Plane.of(np.asarray(pic), "bilinear")
        if pic.mode == "P":
            return U8Plane.of(np.asarray(pic), "nearest")
        if pic.mode == "1":
            return U8Plane.of(np.asarray(pic.convert("L")), "nearest")
        raise ValueError(f"image mode {pic.mode!r}: the device pipeline takes single-band 8-bit "
                         f"images ('L', 'P' or '1'; this one has bands {pic.getbands()})")

    def __call__(self, img, mask):
        return self._plane(img), self._plane(mask)


def u8_collate(batch):
    """Keep variable-size uint8 planes as lists (resized on the device)."""
    return [b[0] for b in batch], [b[1] for b in batch]


class DeviceResizeLoader:
    """Wraps a DataLoader of uint8 (image, mask) lists; yields (N, 1, H, W) fp32 device
    batches resized + scaled on the GPU exactly like Resize + ToTensor."""

    def __init__(self, loader, size, device="cuda"):
        from unet_hip import GpuResizeToTensor
        self.loader = loader
        self.pipe = GpuResizeToTensor(size, device)

    def __len__(self):
        return len(self.loader)

    @property
    def batch_sampler(self):
        return self.loader.batch_sampler

    def __iter__(self):
        for batch in self.loader:
            yield None if batch is None else self.pipe(*batch)
