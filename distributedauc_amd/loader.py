"""Synthetic ImageNet-shaped data, generated on the device.

The reference reads ImageNet through torchvision (main.py:94-117) with a
4-worker host DataLoader and copies every batch to the GPU (main.py:285-286).
This build has no dataset and no network, so training data is synthetic with
ImageNet's shape: a label per sample index (class 0..num_classes-1) and
images generated directly in HBM (N(0,1) noise plus a small class-dependent
signal, so the AUC actually moves). Only the int64 label indices cross PCIe,
through pinned memory and non-blocking copies.

The signal is +-``signal`` on channel 0 by class. With ``flip`` > 0 a fixed fraction of the
samples (chosen by a hash of the sample index, so an image keeps its sign in every epoch and on
every rank) carries the OTHER class's sign: no model can see through it, so the best achievable
test AUC is 1 - flip (a score that only reads the sign) instead of 1, and a trained model's AUC
lands between chance and that ceiling (bench.py's in-training evaluation).
"""
from __future__ import annotations

from typing import Iterator, Sequence

import numpy as np
import torch

from .data_partitioner import IMAGENET_LEN, IMAGENET_NEG


def imagenet_like_labels(n: int = IMAGENET_LEN, num_classes: int = 1000, split_index: int = 499,
                         pos_ratio: float | None = None, seed: int = 0) -> np.ndarray:
    """Class index per sample.

    With ``pos_ratio=None`` and n == 1281167 the labels are sorted by class like the
    ImageNet train folder, consistent with the index ranges data_partitioner.py
    hard-codes (negatives 0..642288 <= split_index 499). Otherwise classes are
    drawn so that a fraction ``pos_ratio`` is above ``split_index``.
    """
    if pos_ratio is None and n == IMAGENET_LEN and split_index == 499 and num_classes == 1000:
        i = np.arange(n, dtype=np.int64)
        n_neg = IMAGENET_NEG[1]
        neg_cls = i * 500 // n_neg
        pos_cls = 500 + (i - n_neg) * 500 // (n - n_neg)
        return np.where(i < n_neg, neg_cls, pos_cls).astype(np.int64)
    if pos_ratio is None:
        pos_ratio = (num_classes - 1 - split_index) / num_classes
    rng = np.random.default_rng(seed)
    is_pos = rng.random(n) < pos_ratio
    neg_cls = rng.integers(0, split_index + 1, size=n)
    pos_cls = rng.integers(split_index + 1, num_classes, size=n)
    return np.where(is_pos, pos_cls, neg_cls).astype(np.int64)


def flipped(indices: np.ndarray, flip: float) -> np.ndarray:
    """Which samples carry the other class's sign: a multiplicative hash of the sample index
    (Knuth's 2654435761), below ``flip`` * 2^32 -- a fixed fraction ``flip`` of the indices."""
    if flip <= 0:
        return np.zeros(len(indices), bool)
    h = (np.asarray(indices, dtype=np.uint64) * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)
    return h < np.uint64(int(flip * 2 ** 32))


def signal_auc_ceiling(indices: np.ndarray, labels: np.ndarray, split_index: int, flip: float) -> float:
    """The exact AUC of the best possible score on these samples -- the sign each image carries
    (1 for +, 0 for -, ties counted half as sklearn does): 1 - flip in expectation."""
    pos = np.asarray(labels)[np.asarray(indices)] > split_index
    plus = pos ^ flipped(indices, flip)
    P, N = int(pos.sum()), int((~pos).sum())
    if P == 0 or N == 0:
        return float("nan")
    a, b = int((plus & pos).sum()), int((plus & ~pos).sum())  # + signs among positives / negatives
    wins = a * (N - b)
    ties = a * b + (P - a) * (N - b)
    return (2 * wins + ties) / (2 * P * N)


class SyntheticImageNet:
    """Index -> (image spec, class label). Images are materialised per batch on the device."""

    def __init__(self, labels: np.ndarray, image_size: int = 224, split_index: int = 499):
        self.labels = np.asarray(labels, dtype=np.int64)
        self.image_size = image_size
        self.split_index = split_index

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        return i, int(self.labels[i])


class DeviceLoader:
    """Infinite iterator of (images [B,3,R,R], labels int64 [B]) on ``device``.

    Epochs reshuffle ``indices`` (like DataLoader(shuffle=True)) with a seeded RNG;
    a final partial batch is kept (drop_last=False, the DataLoader default).
    ``pool`` > 0 pre-generates that many batches once and cycles them, so a timed
    loop reads inputs already resident in HBM. ``dtype``: the images' dtype (bf16 for a bf16
    autocast model: the values its first convolution would cast them to, cast once here instead
    of every step).
    """

    def __init__(self, dataset: SyntheticImageNet, indices: Sequence[int], batch_size: int, device,
                 seed: int = 0, shuffle: bool = True, channels_last: bool = True, signal: float = 0.25,
                 pool: int = 0, drop_last: bool = False, flip: float = 0.0, dtype: torch.dtype = torch.float32):
        self.ds = dataset
        self.indices = np.asarray(indices, dtype=np.int64)
        if self.indices.size == 0:
            raise ValueError("empty partition")
        self.B = int(batch_size)
        self.device = torch.device(device)
        self.seed = seed
        self.shuffle = shuffle
        self.channels_last = channels_last
        self.signal = signal
        self.flip = float(flip)
        self.drop_last = drop_last
        self.dtype = dtype
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self._pool = [self._make(b) for b in self._index_batches(pool)] if pool else None

    def _index_batches(self, limit: int | None = None) -> Iterator[np.ndarray]:
        epoch, made = 0, 0
        while True:
            order = self.indices
            if self.shuffle:
                order = np.random.default_rng(self.seed + epoch).permutation(self.indices)
            stop = len(order) - (len(order) % self.B if self.drop_last else 0)
            for s in range(0, stop, self.B):
                yield order[s:s + self.B]
                made += 1
                if limit is not None and made >= limit:
                    return
            epoch += 1

    def _make(self, idx: np.ndarray):
        R = self.ds.image_size
        lab_host = torch.from_numpy(self.ds.labels[idx])
        if self.device.type == "cuda":
            lab_host = lab_host.pin_memory()
        labels = lab_host.to(self.device, non_blocking=True)
        x = torch.randn((len(idx), 3, R, R), generator=self.gen, device=self.device, dtype=torch.float32)
        if self.signal:
            if self.flip > 0:
                plus = (self.ds.labels[idx] > self.ds.split_index) ^ flipped(idx, self.flip)
                sign = torch.from_numpy(np.where(plus, 1.0, -1.0).astype(np.float32)).to(self.device)
            else:
                sign = torch.where(labels > self.ds.split_index, 1.0, -1.0).to(torch.float32)
            x[:, 0].add_(sign.view(-1, 1, 1), alpha=self.signal)
        if self.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        if self.dtype != torch.float32:
            x = x.to(self.dtype)  # preserves the memory format
        return x, labels

    def __iter__(self):
        if self._pool is not None:
            k = 0
            while True:
                yield self._pool[k % len(self._pool)]
                k += 1
        for idx in self._index_batches():
            yield self._make(idx)


def synthetic_scores(n: int, pos_ratio: float, device, seed: int = 2024) -> tuple[torch.Tensor, torch.Tensor]:
    """The exact-AUC workloads of BASELINE configs[3] / [4]: scores ~ U(0,1) fp32
    and int8 labels +1 with probability ``pos_ratio`` (else -1), drawn in HBM from one seeded
    device generator, so every rank (and every test) that asks for the same (n, p, seed) gets
    the same vectors."""
    g = torch.Generator(device=device).manual_seed(seed)
    s = torch.rand(n, generator=g, device=device)
    y = torch.where(torch.rand(n, generator=g, device=device) < pos_ratio, 1, -1).to(torch.int8)
    return s, y
