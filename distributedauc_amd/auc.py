"""Exact AUC on the GPU: stable split + integer pair count, sharded over ranks.

Replaces ``AUC(label, scores)`` (main.py:79-81), i.e. sklearn
``roc_curve(label, scores, pos_label=1)`` followed by ``auc``. sklearn's area is
(2W + T) / (2PN) where W counts (positive, negative) pairs ordered correctly and
T counts tied pairs; the kernels here compute W and T as exact integers, so the
counts are bit-exact against the reference on identical scores and the returned
float is within a few ulp of sklearn's trapezoid sum.

Two exact methods give the same integers: ``method="pairs"`` runs the LDS-tiled
pair-count kernel (O(P*N), the north-star kernel) and ``method="sort"`` (default)
compacts the positives, builds an LDS count index straight from them (cells of the
score's order-preserving key, no sort) and locates every other score in it
(O(n + P)); tables the index cannot hold (clustered or more than
219,838 positives) take a radix sort + LDS search tree instead.

Sharding (north star): every rank holds the same score vector. The
pair-count method gives rank r the positives [r*P/G, (r+1)*P/G) of the stable
split against ALL negatives, then one all-gather of every rank's 6-word record
(W, T, P, N, non-finite, other): the split's figures must agree. The sort method has
every rank compact the positives of its slice of the labels into a slot,
all-gathers the slots (every rank then holds the whole positive table), builds the
count index from them, counts the next rank's slice of the scores, and all-gathers
the parts' 8-word records (two collectives, one host read, no host synchronisation
before the read); each record carries a check of the queried slice's labels
against the slot the next rank compacted from it, and of the length every slot was
built for. The result does not depend on G. A mismatch raises RuntimeError on every
rank together, after the collective; the scores are not compared across ranks.

Error behaviour mirrors sklearn 1.7.2's roc_curve(pos_label=1): non-finite scores
raise ValueError; every label other than 1 is a negative, whatever the number of
distinct label values (sklearn accepts a "multiclass" y_true when pos_label is
given: {-1, 0, 1} scores as {negative, negative, positive}); non-integer float
labels raise ValueError ("continuous format is not supported"); a single class
returns NaN with a warning. The kernels count the labels outside {-1, 1}
("other"), which is reported, not an error.
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
    if y.dtype.is_floating_point and y.numel() and not bool((y == y.round()).all()):
        # sklearn's type_of_target: non-integer float labels are "continuous" (_ranking.py:826's check)
        raise ValueError("continuous format is not supported")
    if y.dtype not in (torch.int8, torch.int32, torch.int64):
        y = y.to(torch.int64)
    return y.contiguous(), s


class ExactAUC:
    """Exact AUC evaluator; sharded over a process group when world > 1."""

    # Below this many scores the sort method does not shard: every rank evaluates the whole vector
    # (same integers, no collective). Sharding saves (G-1)/G of the compaction and of the query pass
    # (0.15 ms on one GPU at 2^24) but every rank still builds the count index from all the gathered
    # positives (~30 us) and pays two all-gathers and their launches, so it pays from ~2^24 scores.
    SHARD_MIN = 1 << 24

    def __init__(self, group=None, world: int = 1, rank: int = 0, variant: int = 0, reduce: bool = True,
                 method: str = "sort", shard_min: int | None = None, collective: bool | None = None):
        if method not in ("sort", "pairs"):
            raise ValueError("method must be 'sort' (radix sort + search) or 'pairs' (pair-count kernel)")
        self.group = group
        self.world = world
        self.rank = rank
        # collective: take the sharded path with its collectives (default: world > 1). True at world
        # 1 is the RCCL rehearsal: the world > 1 code path on a one-rank process group
        self.collective = world > 1 if collective is None else bool(collective)
        self.variant = variant
        self.reduce = reduce  # False: return only this rank's share (no collective)
        self.method = method
        self.shard_min = self.SHARD_MIN if shard_min is None else int(shard_min)
        self.last_mode = None  # "single", "replicated" or "sharded" (the last call's)
        self._part_counts: dict = {}  # device -> int64 [8 (1 + world)]: this part's record + the gathered ones
        self._slots: dict = {}        # (device, n) -> (this rank's slot, the gathered slots)

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
        if self.method == "sort":
            return self._counts_sort(y, s)
        self.last_mode = "sharded" if self.collective else "single"
        # the pair-count method: a stable split, so every rank sees the positives in the same order
        # and positive blocks shard
        pos, neg, stats = ops.split_scores(s, y)
        P, N, nonfinite, other = (int(v) for v in stats.tolist())
        wt = torch.zeros(3, dtype=torch.int64, device=s.device)
        if P and N and not nonfinite:
            lo, hi = self.rank * P // self.world, (self.rank + 1) * P // self.world
            if hi > lo:
                ops.pair_count(pos[lo:hi], neg[:N], wt, variant=self.variant)
        if self.collective and self.reduce:
            # one all-gather of every rank's (W, T, P, N, non-finite, other): the split's figures
            # must agree (ranks holding different test sets raise together), and no rank raises
            # before the collective, so a bad input cannot leave the others waiting in it
            mine = torch.cat((wt[:2], stats.to(device=wt.device, dtype=torch.int64)))
            gathered = torch.empty(6 * self.world, dtype=torch.int64, device=wt.device)
            dist.all_gather_into_tensor(gathered, mine, group=self.group)
            vals = gathered.view(self.world, 6).tolist()
            if len({tuple(v[2:]) for v in vals}) != 1:
                raise RuntimeError("ExactAUC: the ranks' parts disagree on the test set (positives, non-finite or "
                                   "label counts): every rank must pass the same scores and labels")
            W, T = sum(v[0] for v in vals), sum(v[1] for v in vals)
        else:
            W, T, _ = (int(v) for v in wt.tolist())
        if nonfinite:
            raise ValueError("Input y_score contains NaN or infinity.")
        return {"wins": W, "ties": T, "P": P, "N": N, "other": other}

    def _counts_sort(self, y: torch.Tensor, s: torch.Tensor) -> dict:
        """The sort method. One GPU (or a vector below ``shard_min``, which every rank evaluates
        whole: same integers, no collective): ONE blocking C call (dauc_auc_eval_counts). Over
        ranks: every rank compacts its slice of the labels into a slot (dauc_auc_eval_compact_part),
        one all-gather of the slots, every rank builds the index from the gathered positives and
        counts the NEXT rank's slice of the scores (dauc_auc_eval_query_part), one all-gather of the
        parts' 8-word records, and ONE host read of the gathered records. P and the label counts
        come from the gathered slots, so they are the same on every rank by construction; what the
        ranks could disagree on is checked through record word 4 instead: every rank's query pass
        compares the positives its own labels give over the next rank's slice with the slot that
        rank compacted from it, and every build compares the length each slot was built for. A mismatch raises RuntimeError on every rank together, after the collective
        (the slot size does not depend on n, so differing lengths cannot desynchronise the gather).
        The scores are not compared across ranks (that would take a second pass over them). With reduce=False each rank evaluates
        its part against all the positives itself (no collective, no check)."""
        if not self.collective or (self.reduce and s.numel() < self.shard_min):
            self.last_mode = "single" if not self.collective else "replicated"
            W, T, P, N, nonfinite, other = ops.auc_eval_counts(s, y)
            if nonfinite:
                raise ValueError("Input y_score contains NaN or infinity.")
            return {"wins": W, "ties": T, "P": P, "N": N, "other": other}
        self.last_mode = "sharded"
        n = s.numel()
        rec = self._part_counts.get(s.device)
        if rec is None:
            rec = self._part_counts[s.device] = torch.zeros(8 * (self.world + 1), dtype=torch.int64, device=s.device)
        mine, gathered = rec[:8], rec[8:]
        if not self.reduce:
            # no collective: this rank's part with the table built from ALL the positives itself
            ops.auc_eval_enqueue(s, y, self.rank, self.world, out=mine)
            vals = [mine.tolist()]
        else:
            # each rank compacts only its slice of the labels; one all-gather of the slots gives
            # every rank the whole positive table; each rank counts its query range; one
            # all-gather of the 8-word records (no whole-vector pass per rank)
            slots = self._slots_of(s.device, n)
            nb = ops.auc_slot_bytes(n, self.world)
            ops.auc_eval_compact_part(s, y, self.rank, self.world, slots[0])
            dist.all_gather_into_tensor(slots[1], slots[0], group=self.group)
            ops.auc_eval_query_part(s, y, self.rank, self.world, slots[1][: nb * self.world], out=mine)
            dist.all_gather_into_tensor(gathered, mine, group=self.group)
            vals = gathered.view(self.world, 8).tolist()  # the one host synchronisation
            check = [v[4] & 0xFFFFFFFFFFFFFFFF for v in vals]
            if any(c >> 32 for c in check):
                raise RuntimeError("ExactAUC: the ranks passed test sets of different lengths: every rank must "
                                   "pass the same scores and labels")
            if any(c & 0xFFFFFFFF for c in check):
                raise RuntimeError("ExactAUC: the ranks' parts disagree on the test set (the labels of a slice "
                                   "differ between the rank that compacted it and the rank that queried it): every "
                                   "rank must pass the same scores and labels")
        P, nonfinite, other = vals[0][3], vals[0][5], vals[0][6]
        verdicts = {v[7] for v in vals} - {0}
        # every label other than 1 is a negative (pos_label=1), and word 4 above has checked that
        # every rank holds this n and these labels: N = n - P on every rank
        N = n - P
        if nonfinite or sum(v[2] for v in vals):
            raise ValueError("Input y_score contains NaN or infinity.")
        if P == 0 or N == 0:
            return {"wins": 0, "ties": 0, "P": P, "N": N, "other": other}
        if 2 in verdicts:
            if self.reduce and P <= N:
                # the gathered slots still hold every positive (unless a slot overflowed): each rank
                # sorts them and counts its own slice (tie-heavy tables: the distinct-key index), one
                # more all-gather of the records -- no whole-vector compaction on any rank
                ops.auc_eval_query_part_sorted(s, y, self.rank, self.world, slots[1][: nb * self.world], P, out=mine)
                dist.all_gather_into_tensor(gathered, mine, group=self.group)
                vals2 = gathered.view(self.world, 8).tolist()
                if all(v[7] == 1 for v in vals2):
                    if sum(v[2] for v in vals2):
                        raise ValueError("Input y_score contains NaN or infinity.")
                    return {"wins": sum(v[0] for v in vals2), "ties": sum(v[1] for v in vals2), "P": P, "N": N,
                            "other": other}
            return dict(self._counts_sort_sorted_path(y, s), other=other)
        return {"wins": sum(v[0] for v in vals), "ties": sum(v[1] for v in vals), "P": P, "N": N, "other": other}

    def _slots_of(self, device, n: int):
        """(this rank's slot, the gathered slots) for n scores: uint8 device buffers, 256-byte
        aligned (auc_slot_bytes(n, world) bytes per rank), cached per (device, n)."""
        key = (device, n)
        got = self._slots.get(key)
        if got is None:
            nb = ops.auc_slot_bytes(n, self.world)
            # torch allocations are 256-byte aligned; nb is a multiple of 256
            got = self._slots[key] = (torch.empty(nb, dtype=torch.uint8, device=device),
                                      torch.empty(nb * self.world, dtype=torch.uint8, device=device))
        return got

    def _counts_sort_sorted_path(self, y: torch.Tensor, s: torch.Tensor) -> dict:
        """A table the count index cannot hold (more than 219,838 positives, or clustered ones):
        every rank runs the blocking part (the sorted path, its own whole compaction) and one
        all-gather of the parts' (W, T, #non-finite queried, P) sums the counts; the parts' P must
        agree. Every rank reached here with the same verdicts, so all take this branch."""
        wt = torch.zeros(4, dtype=torch.int64, device=s.device)
        W, T, P, N, nonfinite, other, qbad = ops.auc_eval_counts_part(s, y, self.rank, self.world, wt)
        if self.reduce:
            wt[3] = P
            got = torch.empty(4 * self.world, dtype=torch.int64, device=s.device)
            dist.all_gather_into_tensor(got, wt, group=self.group)
            vals = got.view(self.world, 4).tolist()
            if len({v[3] for v in vals}) != 1:
                raise RuntimeError("ExactAUC: the ranks' parts disagree on the test set (positives): every rank "
                                   "must pass the same scores and labels")
            W, T, qbad = sum(v[0] for v in vals), sum(v[1] for v in vals), sum(v[2] for v in vals)
        if qbad:
            raise ValueError("Input y_score contains NaN or infinity.")
        return {"wins": W, "ties": T, "P": P, "N": N}

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
