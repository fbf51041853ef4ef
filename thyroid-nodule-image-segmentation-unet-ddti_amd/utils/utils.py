"""Host-side bookkeeping the Trainer needs (mirror of the reference's utils/utils.py).

Off the hot path.  Same public names and semantics as the reference:
Config (:15-45), set_seed (:47-51), AverageMeter (:53-70), create_logger (:125-171),
EarlyStopping (:173-202) and the binary-mask metrics (:225-251).  The metrics also have
``*_from_counts`` forms that take the device-side confusion counts of
``unet_mask_counts`` (so a whole epoch's predictions never travel to the host) and give
the same numbers as the array forms.
"""
import logging
import os
import random
from datetime import datetime, timedelta, timezone

import numpy as np
import torch
import yaml


class Config:
    """argparse namespace -> attributes + experiments/<model>_<UTC+8 stamp>/ tree + YAML dump."""

    def __init__(self, args, base_dir="experiments", stamp=None):
        for k, v in vars(args).items():
            setattr(self, k, v)
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        stamp = stamp or self.make_stamp()
        self.base_dir = base_dir
        self.cfg_dir = os.path.join(base_dir, f"{self.model_type}_{stamp}")
        self.model_dir = os.path.join(self.cfg_dir, "models")
        self.log_dir = os.path.join(self.cfg_dir, "log")
        self.result_dir = os.path.join(self.cfg_dir, "result")
        for d in (self.cfg_dir, self.model_dir, self.log_dir, self.result_dir):
            os.makedirs(d, exist_ok=True)
        if not (torch.distributed.is_available() and torch.distributed.is_initialized()) \
                or torch.distributed.get_rank() == 0:
            self._dump()

    @staticmethod
    def make_stamp():
        return (datetime.now(timezone.utc) + timedelta(hours=8)).strftime("%Y%m%d_%H%M%S")

    def _dump(self):
        with open(os.path.join(self.cfg_dir, "config.yaml"), "w") as f:
            yaml.safe_dump({k: (str(v) if isinstance(v, torch.device) else v)
                            for k, v in self.__dict__.items() if not k.startswith("_")}, f)


def set_seed(seed):
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)


class AverageMeter:
    def __init__(self):
        self.reset()

    def reset(self):
        self.val = self.avg = self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


def create_logger(filename):
    """Console (INFO) + file (DEBUG) logger with UTC+8 timestamps."""
    def utc8(*_):
        return (datetime.now(tz=timezone.utc) + timedelta(hours=8)).timetuple()

    logger = logging.getLogger(filename)
    logger.setLevel(logging.DEBUG)
    fmt = logging.Formatter("%(asctime)s - %(levelname)s - %(message)s")
    fmt.converter = utc8
    if not logger.handlers:
        ch = logging.StreamHandler()
        ch.setLevel(logging.INFO)
        ch.setFormatter(fmt)
        fh = logging.FileHandler(filename)
        fh.setLevel(logging.DEBUG)
        fh.setFormatter(fmt)
        logger.addHandler(ch)
        logger.addHandler(fh)
    return logger


class EarlyStopping:
    """Stops after `patience` calls without improvement of -val_loss by more than delta."""

    def __init__(self, logger, patience=10, delta=0):
        self.patience, self.delta, self.logger = patience, delta, logger
        self.counter = 0
        self.best_score = None
        self.early_stop = False
        self.val_loss_min = np.inf

    def __call__(self, val_loss, model):
        score = -val_loss
        if self.best_score is None or score >= self.best_score + self.delta:
            if self.best_score is not None:
                self.counter = 0
            self.logger.info(f"--Validation loss decreased ({self.val_loss_min:.6f} --> {val_loss:.6f}).")
            self.best_score = score
            self.val_loss_min = val_loss
        else:
            self.counter += 1
            self.logger.info(f"--EarlyStopping counter: {self.counter} out of {self.patience}")
            if self.counter >= self.patience:
                self.early_stop = True


# ---------------------------------------------------------------- metrics
def calculate_iou(pred, target):
    p, t = pred.astype(bool), target.astype(bool)
    return np.logical_and(p, t).sum() / np.logical_or(p, t).sum()


def calculate_acc(pred, target):
    return (pred.astype(int) == target.astype(int)).sum() / pred.size


def calculate_precision_recall_f1(pred, target):
    p, t = pred.astype(int), target.astype(int)
    TP = np.logical_and(p == 1, t == 1).sum()
    FP = np.logical_and(p == 1, t == 0).sum()
    FN = np.logical_and(p == 0, t == 1).sum()
    return _prf1(TP, FP, FN)


def _prf1(TP, FP, FN):
    precision = TP / (TP + FP) if TP + FP > 0 else 0.0
    recall = TP / (TP + FN) if TP + FN > 0 else 0.0
    f1 = 2 * precision * recall / (precision + recall) if precision + recall > 0 else 0.0
    return precision, recall, f1


def metrics_from_counts(counts):
    """counts = [TP, FP, FN, TN, I_bool, U_bool] (unet_mask_counts) -> the epoch metrics of
    utils/trainer.py:104-107 computed by the reference on concatenated host arrays."""
    TP, FP, FN, TN, I, U = [int(c) for c in counts]
    total = TP + FP + FN + TN
    acc = (TP + TN) / total
    precision, recall, f1 = _prf1(TP, FP, FN)
    iou = I / U if U else float("nan")
    return acc, precision, recall, f1, iou


def global_metrics_from_counts(counts, eps=1e-8):
    """Global test metrics of utils/trainer.py:232-250 (targets cast to uint8)."""
    TP, FP, FN, TN = [int(c) for c in counts[:4]]
    ACC = (TP + TN) / (TP + TN + FP + FN + eps)
    P = TP / (TP + FP + eps)
    R = TP / (TP + FN + eps)
    F1 = 2 * P * R / (P + R + eps)
    IoU = TP / (TP + FP + FN + eps)
    return dict(TP=TP, FP=FP, FN=FN, TN=TN, ACC=ACC, Precision=P, Recall=R, F1=F1, IoU=IoU)
