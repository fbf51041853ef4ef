"""CLI entry (mirror of the reference's main.py:17-161) on the HIP UNet path.

Same flags as the reference (``--dataset_path``, ``--checkpoint_path``, ``--bce_ratio`` ...
``--use_data_parallel``), with three additions: ``--model_type`` picks the network
(``ResUNet``: models/mod.py:88-131, what the reference hard-codes at main.py:120-122;
``ModUNet``: models/mod.py:9-66; ``UNet``: models/model.py, the BASELINE network and the
default here; ``--base_filters`` / ``--depth`` for the mod.py ones, default 64 / 5 as
there), ``--mode {train,test,both}`` replaces the commented-out
``trainer.train()`` / hard-wired ``trainer.test()`` (:156-157), and ``--synthetic N`` runs
on N synthetic samples per split when the DDTI images are not on disk.

Multi-GPU: launch one process per GPU, e.g.
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 main.py --mode train ...
(RCCL backend; replaces nn.DataParallel of utils/trainer.py:28-30).
"""
import argparse
import logging
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

from data.data_loader import (DataParallelShardSampler, DecodeU8, DeviceResizeLoader,  # noqa: E402
                              MedicalDataset, SyntheticSegmentation, create_dataloader,
                              dp_collate, u8_collate)
from models.mod import ResUNet  # noqa: E402
from models.mod import UNet as ModUNet  # noqa: E402
from models.model import UNet  # noqa: E402
from utils.trainer import Trainer  # noqa: E402
from utils.transforms import Compose, Resize, ToTensor, build_train_transform  # noqa: E402
from utils.utils import Config, create_logger, set_seed  # noqa: E402


def _flag(v):
    # the reference uses type=bool (main.py:59-60), which turns any string into True
    return bool(v)


def get_parser(argv=None):
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("--dataset_path", default="data/dataset", type=str)
    p.add_argument("--dataset", default="DDTI", type=str)
    p.add_argument("--checkpoint_path", default="", type=str)
    p.add_argument("--config_path", default=None, type=str)
    p.add_argument("--p_crop", default=0, type=float)
    for f in ("--use_elastic", "--use_speckle", "--use_tgc", "--use_clahe", "--use_mixup"):
        p.add_argument(f, action="store_true")
    p.add_argument("--mixup_alpha", type=float, default=0.2)
    p.add_argument("--mixup_prob", type=float, default=0.3)
    p.add_argument("--model_type", default="UNet", type=str, help="UNet | ModUNet | ResUNet")
    p.add_argument("--base_filters", default=64, type=int, help="ModUNet / ResUNet (mod.py:13)")
    p.add_argument("--gpu_transforms", action="store_true",
                   help="decode on the host, Resize + ToTensor on the GPU (bit-identical)")
    p.add_argument("--depth", default=5, type=int, help="ModUNet / ResUNet (mod.py:14)")
    p.add_argument("--bce_ratio", type=float, default=1)
    p.add_argument("--dice_ratio", type=float, default=0)
    p.add_argument("--focal_ratio", type=float, default=1)
    p.add_argument("--boundary_ratio", type=float, default=0)
    p.add_argument("--num_workers", default=4, type=int)
    p.add_argument("--epochs", type=int, default=10000)
    p.add_argument("--batch_size", default=16, type=int)
    p.add_argument("--lr", type=float, default=1e-5)
    p.add_argument("--weight_decay", type=float, default=1e-2)  # unused, as in the reference
    p.add_argument("--save_interval", default=20, type=int)
    p.add_argument("--early_stop_patience", default=50, type=int)
    p.add_argument("--alpha", type=float, default=2)
    p.add_argument("--use_data_parallel", type=_flag, default=True)
    p.add_argument("--use_amp_autocast", type=_flag, default=False)
    p.add_argument("--mode", choices=["train", "test", "both"], default="test")
    p.add_argument("--image_size", type=int, default=512)
    p.add_argument("--synthetic", type=int, default=0, help="synthetic samples per split")
    return p.parse_args(argv)


def main(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not torch.distributed.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    set_seed(seed=42)
    rank = torch.distributed.get_rank() if world > 1 else 0
    if rank:
        # per-rank host augmentation streams (utils/transforms.py draws from random / numpy
        # in the main process when num_workers == 0): otherwise every shard would get rank 0's
        # Flip / Rotate / ... sequence.  torch's stream stays shared (identical model init;
        # parameters are broadcast from rank 0 anyway) and the mixup draws come from rank 0.
        random.seed(42 + rank)
        np.random.seed(42 + rank)
    stamp = [None]
    if world > 1:  # one experiments/<model>_<stamp>/ tree for the job: rank 0's
        stamp = [Config.make_stamp()] if rank == 0 else [None]
        torch.distributed.broadcast_object_list(stamp, src=0)
    config = Config(args, stamp=stamp[0])
    if torch.cuda.is_available():
        config.device = torch.device("cuda", torch.cuda.current_device())
    if rank == 0:
        logger = create_logger(os.path.join(config.log_dir, "train_log.log"))
    else:  # one writer of the shared log file (the Trainer also logs from rank 0 only)
        logger = logging.getLogger(f"unet_hip.rank{rank}")
        logger.addHandler(logging.NullHandler())
        logger.propagate = False
    if args.model_type not in ("UNet", "ModUNet", "ResUNet"):
        raise SystemExit(f"model_type {args.model_type!r}: the HIP path has UNet (models/model.py), "
                         "ModUNet and ResUNet (models/mod.py)")

    S = args.image_size
    gpu_tf = args.gpu_transforms and not args.synthetic
    if args.synthetic:
        splits = [SyntheticSegmentation(args.synthetic, S, seed=s) for s in range(3)]
    else:
        # main.py:99-100: augmentations on the training split only
        tf = DecodeU8() if gpu_tf else Compose([Resize((S, S)), ToTensor()])
        train_tf = build_train_transform(config, (S, S), tail=[DecodeU8()] if gpu_tf else None)
        root = config.dataset_path
        splits = [MedicalDataset(os.path.join(root, d), os.path.join(root, d + "_mask"),
                                 train_tf if d == "train" else tf)
                  for d in ("train", "val", "test")]
    loaders = []
    for i, ds in enumerate(splits):
        kw = dict(batch_size=config.batch_size, num_workers=config.num_workers)
        if gpu_tf:
            kw["collate_fn"] = u8_collate
        if world > 1:
            # nn.DataParallel's split of every global batch (utils/trainer.py:28-30):
            # --batch_size stays the GLOBAL batch, as in the reference
            bs = DataParallelShardSampler(len(ds), config.batch_size, i != 1, rank, world, seed=42)
            # per-rank worker seeds (the sampler's shared order seed is separate): DataLoader
            # derives each worker's random / numpy / torch seeds from this generator
            dl = torch.utils.data.DataLoader(ds, batch_sampler=bs, num_workers=config.num_workers,
                                             collate_fn=dp_collate(u8_collate if gpu_tf else None),
                                             generator=torch.Generator().manual_seed(42 + rank))
        elif gpu_tf:
            dl = torch.utils.data.DataLoader(ds, shuffle=(i != 1), **kw)
        else:
            dl = create_dataloader(ds, config, shuffle=(i != 1))
        loaders.append(DeviceResizeLoader(dl, (S, S), config.device) if gpu_tf else dl)

    if args.model_type == "ResUNet":
        model = ResUNet(base_filters=args.base_filters, depth=args.depth)
    elif args.model_type == "ModUNet":
        model = ModUNet(base_filters=args.base_filters, depth=args.depth)
    else:
        model = UNet()
    if config.checkpoint_path and os.path.isfile(config.checkpoint_path):
        model.load_state_dict(torch.load(config.checkpoint_path, weights_only=True))
    n = sum(p.numel() for p in model.parameters() if p.requires_grad)
    logger.info(f"Model: {config.model_type} | Trainable params: {n / 1e6:.2f}M ({n:,})")
    if rank == 0:
        print(f"[PARAMS] {config.model_type},{n}")

    trainer = Trainer(config, tuple(loaders), logger, model)
    if args.mode in ("train", "both"):
        trainer.train()
    if args.mode in ("test", "both"):
        trainer.test()


if __name__ == "__main__":
    main(get_parser())
