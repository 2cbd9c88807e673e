"""Exact AUC on the GPU: stable split + integer pair count, sharded over ranks.

Replaces ``AUC(label, scores)`` (main.py:79-81), i.e. sklearn
``roc_curve(label, scores, pos_label=1)`` followed by ``auc``. sklearn's area is
(2W + T) / (2PN) where W counts (positive, negative) pairs ordered correctly and
T counts tied pairs; the kernels here compute W and T as exact integers, so the
counts are bit-exact against the reference on identical scores and the returned
float is within a few ulp of sklearn's trapezoid sum.

Two exact methods give the same integers: ``method="pairs"`` runs the LDS-tiled
pair-count kernel (O(P*N), the north-star kernel) and ``method="sort"`` (default)
radix-sorts the smaller class and locates every score of the larger class in it
through an LDS search tree (O(M log M + L log M)).

Sharding (north star): every rank holds the same score vector. The
pair-count method gives rank r the positives [r*P/G, (r+1)*P/G) of the stable
split against ALL negatives; the sort method has rank r compact the positives of
its index slice (all ranks then all-gather them, in order) and stream its slice
of the scores through the search over ALL positives. One int64 [3] all-reduce
sums (W, T, non-finite); the result does not depend on G.

Error behaviour mirrors sklearn: non-finite scores raise ValueError; labels
with more than two distinct values raise ValueError; a single class returns NaN
with a warning.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch
import torch.distributed as dist

from . import ops


class UndefinedMetricWarning(UserWarning):
    """Same meaning as sklearn.exceptions.UndefinedMetricWarning."""


def _as_device_pair(label, scores, device):
    dev = torch.device(device) if device is not None else None
    if isinstance(scores, torch.Tensor):
        s = scores.detach()
        if dev is None:
            dev = s.device if s.device.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
        s = s.to(dev, torch.float32).reshape(-1).contiguous()
    else:
        if dev is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        s = torch.as_tensor(np.asarray(scores, dtype=np.float32).reshape(-1), device=dev)
    if isinstance(label, torch.Tensor):
        y = label.detach().to(dev).reshape(-1)
    else:
        y = torch.as_tensor(np.asarray(label).reshape(-1), device=dev)
    if y.dtype not in (torch.int8, torch.int32, torch.int64):
        y = y.to(torch.int64)
    return y.contiguous(), s


class ExactAUC:
    """Exact AUC evaluator; sharded over a process group when world > 1."""

    # Below this many scores the sort method does not shard: every rank evaluates the whole vector
    # (same integers, no collective). Sharding saves ~5 ns per query per rank but costs two small
    # all-gathers with a host sync and an all-reduce (~150-200 us), so it pays from ~2^25 scores.
    SHARD_MIN = 1 << 25

    def __init__(self, group=None, world: int = 1, rank: int = 0, variant: int = 0, reduce: bool = True,
                 method: str = "sort", shard_min: int | None = None):
        if method not in ("sort", "pairs"):
            raise ValueError("method must be 'sort' (radix sort + search) or 'pairs' (pair-count kernel)")
        self.group = group
        self.world = world
        self.rank = rank
        self.variant = variant
        self.reduce = reduce  # False: return only this rank's share (no collective)
        self.method = method
        self.shard_min = self.SHARD_MIN if shard_min is None else int(shard_min)
        self.last_mode = None  # "single", "replicated" or "sharded" (the last call's)

    def counts(self, label, scores, device=None) -> dict:
        """Exact {wins, ties, P, N} (Python ints). One host sync for the split sizes."""
        if (device is None and isinstance(scores, torch.Tensor) and isinstance(label, torch.Tensor)
                and scores.is_cuda and scores.dtype == torch.float32 and scores.dim() == 1
                and scores.is_contiguous() and label.device == scores.device and label.dim() == 1
                and label.dtype in (torch.int8, torch.int32, torch.int64) and label.is_contiguous()
                and not scores.requires_grad):
            y, s = label, scores  # already what the kernels read: no conversion ops
        else:
            y, s = _as_device_pair(label, scores, device)
        if y.numel() != s.numel():
            raise ValueError(f"Found input variables with inconsistent numbers of samples: {[y.numel(), s.numel()]}")
        if self.method == "sort" and (self.world == 1 or (self.reduce and s.numel() < self.shard_min)):
            # one GPU (or a vector too small to be worth sharding: every rank evaluates all of it):
            # the whole evaluation is one blocking C call (same stages, no host work between)
            self.last_mode = "single" if self.world == 1 else "replicated"
            W, T, P, N, nonfinite, other = ops.auc_eval_counts(s, y)
            if nonfinite:
                raise ValueError("Input y_score contains NaN or infinity.")
            if other and torch.unique(y).numel() > 2:
                raise ValueError("multiclass format is not supported")
            return {"wins": W, "ties": T, "P": P, "N": N}
        self.last_mode = "sharded" if self.world > 1 else "single"
        if self.method == "pairs":
            # stable split: every rank sees the positives in the same order, so positive blocks shard
            pos, neg, stats = ops.split_scores(s, y)
            P, N, nonfinite, other = (int(v) for v in stats.tolist())
        elif self.world > 1 and self.reduce:
            # the sort method over ranks: each rank compacts the positives of its own index slice,
            # then every rank gathers all of them (in index order, so every rank holds the same list)
            pos, (P, N, nonfinite, other) = self._compact_sharded(s, y)
        else:
            # the sort method reads the negatives in place: only the labels and the positives' scores
            # are read here; the negatives' finiteness is checked by the query kernel
            pos, stats = ops.compact_positives(s, y)
            P, N, nonfinite, other = (int(v) for v in stats.tolist())
        if nonfinite:
            raise ValueError("Input y_score contains NaN or infinity.")
        if other:
            distinct = torch.unique(y)
            if distinct.numel() > 2:
                raise ValueError("multiclass format is not supported")
        # wins, ties, non-finite queried scores (sort method, P <= N)
        wt = torch.zeros(3, dtype=torch.int64, device=s.device)
        if self.method == "sort" and (P == 0 or N == 0 or P > N):
            # no query pass over the negatives (one class empty) or the negatives are the sorted table:
            # materialise both classes; the split checks every score
            pos, neg, stats = ops.split_scores(s, y)
            if int(stats[2].item()):
                raise ValueError("Input y_score contains NaN or infinity.")
        if P and N:
            if self.method == "pairs":
                # positive-set blocks: every rank compares its block against all negatives
                lo, hi = self.rank * P // self.world, (self.rank + 1) * P // self.world
                if hi > lo:
                    ops.pair_count(pos[lo:hi], neg[:N], wt, variant=self.variant)
            elif P <= N:
                # the sorted table is the (small) positive class on every rank; the negatives are
                # read in place from the full score/label arrays, whose index range is split
                n = s.numel()
                lo, hi = self.rank * n // self.world, (self.rank + 1) * n // self.world
                if hi > lo:
                    ops.auc_counts_sorted_labeled(pos[:P], s, y, lo, hi, wt, nonfinite=wt[2:])
            else:
                # more positives than negatives: the negatives are the sorted table
                lo, hi = self.rank * P // self.world, (self.rank + 1) * P // self.world
                if hi > lo:
                    ops.auc_counts_sorted(pos[lo:hi], neg[:N], wt)
        if self.world > 1 and self.reduce:
            dist.all_reduce(wt, op=dist.ReduceOp.SUM, group=self.group)
        W, T, bad = (int(v) for v in wt.tolist())
        if bad:
            raise ValueError("Input y_score contains NaN or infinity.")
        return {"wins": W, "ties": T, "P": P, "N": N}

    def _compact_sharded(self, s: torch.Tensor, y: torch.Tensor):
        """dauc_compact_positives over this rank's index slice, then an all-gather of the per-rank
        stats (one host sync) and of the positives (padded to the largest share): every rank ends
        with all the positive scores in original order and the global {P, N, non-finite, other}."""
        n, G, r = s.numel(), self.world, self.rank
        lo, hi = r * n // G, (r + 1) * n // G
        if hi > lo:
            pos_r, st_r = ops.compact_positives(s[lo:hi], y[lo:hi])
        else:
            pos_r, st_r = s.new_empty(0), torch.zeros(4, dtype=torch.int64, device=s.device)
        st_all = [torch.empty_like(st_r) for _ in range(G)]
        dist.all_gather(st_all, st_r, group=self.group)
        st = torch.stack(st_all).cpu()
        sizes = st[:, 0].tolist()
        P, N, nonfinite, other = (int(v) for v in st.sum(0).tolist())
        width = max(sizes)
        if width == 0:
            return s.new_empty(0), (P, N, nonfinite, other)
        send = s.new_empty(width)
        send[:sizes[r]] = pos_r[:sizes[r]]
        parts = [torch.empty_like(send) for _ in range(G)]
        dist.all_gather(parts, send, group=self.group)
        return torch.cat([parts[q][:sizes[q]] for q in range(G) if sizes[q]]), (P, N, nonfinite, other)

    @staticmethod
    def from_counts(c: dict) -> float:
        P, N = c["P"], c["N"]
        if P == 0 or N == 0:
            warnings.warn("No negative samples in y_true, false positive value should be meaningless"
                          if N == 0 else
                          "No positive samples in y_true, true positive value should be meaningless",
                          UndefinedMetricWarning, stacklevel=3)
            return float("nan")
        return (2 * c["wins"] + c["ties"]) / (2 * P * N)

    def __call__(self, label, scores, device=None) -> float:
        return self.from_counts(self.counts(label, scores, device))


def AUC(label, scores) -> float:  # noqa: N802 (reference name, main.py:79)
    """Drop-in for main.py:79-81 on the GPU (single rank)."""
    return ExactAUC()(label, scores)
