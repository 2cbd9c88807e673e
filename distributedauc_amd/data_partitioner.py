"""Dataset partitioning across ranks (data_partitioner.py of the reference).

Two modes:

* ``mode="reference"`` reproduces data_partitioner.py:22-90 bit for bit: the
  ImageNet index ranges are hard-coded there (negatives 0..642288, positives
  642290..1281166; index 642289 is never used), shuffled with Python's
  ``random.Random(seed)``, negatives cut to ``neg_keep_ratio``, the union
  shuffled again, and contiguous fractions sliced off. The resulting shards are
  not class-stratified: the positive fraction drifts from rank to rank.
* ``mode="stratified"`` (default for new runs) is imbalance-preserving: it
  shuffles positives and negatives separately (same seeded RNG), applies
  ``neg_keep_ratio`` and gives every partition the same fraction of EACH class,
  so every rank trains at the global positive rate. It needs the labels.
"""
from __future__ import annotations

import random
from typing import Sequence

import numpy as np

IMAGENET_LEN = 1281167
IMAGENET_NEG = (0, 642289)
IMAGENET_POS = (642290, 1281167)


class Partition:
    """A view of ``data`` restricted to ``index`` (data_partitioner.py:5-16)."""

    def __init__(self, data, index):
        self.data = data
        self.index = index

    def __len__(self):
        return len(self.index)

    def __getitem__(self, i):
        return self.data[self.index[i]]


def _slice_fractions(idx: list, sizes: Sequence[float]) -> list[list]:
    n = len(idx)
    out, start = [], 0
    for frac in sizes:
        k = int(frac * n)  # data_partitioner.py:88 (fractions of the kept total)
        out.append(idx[start:start + k])
        start += k
    return out


class DataPartitioner:
    """Split a dataset into ``sizes`` fractions; partition 0 is the test set by convention (main.py:105-108)."""

    def __init__(self, data, sizes: Sequence[float], seed: int = 123, neg_keep_ratio: float = 1.0,
                 mode: str = "reference", labels=None, split_index: int | None = None):
        self.data = data
        self.sizes = list(sizes)
        rng = random.Random()
        rng.seed(seed)
        if mode == "reference":
            neg = list(range(*IMAGENET_NEG))
            pos = list(range(*IMAGENET_POS))
            rng.shuffle(pos)
            rng.shuffle(neg)
            neg = neg[: int(len(neg) * neg_keep_ratio)]
            union = pos + neg
            rng.shuffle(union)
            self.partitions = _slice_fractions(union, self.sizes)
        elif mode == "stratified":
            if labels is None or split_index is None:
                raise ValueError("stratified partitioning needs labels and split_index")
            lab = np.asarray(labels)
            pos = np.flatnonzero(lab > split_index).tolist()
            neg = np.flatnonzero(lab <= split_index).tolist()
            rng.shuffle(pos)
            rng.shuffle(neg)
            neg = neg[: int(len(neg) * neg_keep_ratio)]
            parts_p = _slice_fractions(pos, self.sizes)
            parts_n = _slice_fractions(neg, self.sizes)
            self.partitions = []
            for pp, pn in zip(parts_p, parts_n):
                merged = pp + pn
                rng.shuffle(merged)
                self.partitions.append(merged)
        else:
            raise ValueError(f"unknown partition mode {mode!r}")

    def use(self, partition: int) -> Partition:
        return Partition(self.data, self.partitions[partition])


def partition_sizes(world: int, test_ratio: float) -> list[float]:
    """main.py:105: [test_ratio] + [(1 - test_ratio) / world] * world."""
    return [test_ratio] + [(1 - test_ratio) / world for _ in range(world)]
