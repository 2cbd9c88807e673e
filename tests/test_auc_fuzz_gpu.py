"""Randomised parity sweep of the exact-AUC paths against the C oracle (round 6).

Seeded cases mix the things the structured suites test one at a time: odd lengths (scalar heads and
tails), every label width, label vectors with values outside {-1, 1}, positive ratios from a
handful of positives to a positive majority, and score distributions from spread to tie-heavy
(rounded grids, bf16, a few values, dense clusters of consecutive floats, signed values with +-0).
Each case runs the one-call evaluation (dauc_auc_eval_counts: the slotted count index, or verdict 2
and the sorted path's distinct-key index / tree / split) and the two-step sharded form over a random
number of parts (compact, gather, query, then the sorted slot fallback or the whole-vector path on
verdict 2, exactly as ExactAUC sequences them). Bar: (W, T, P, N) bit-exact against
oracle/auc_oracle.c (sklearn's _binary_clf_curve counts, main.py:79-81); non-finite scores raise.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import coracle

pytestmark = pytest.mark.gpu

N_CASES = 40


def _scores(rng, n: int, kind: str) -> np.ndarray:
    u = rng.random(n, dtype=np.float32)
    if kind == "uniform":
        return u
    if kind == "bf16":
        return torch.from_numpy(u).bfloat16().float().numpy()
    if kind == "grid":
        k = int(rng.choice([3, 10, 100, 1000, 10_000, 30_000]))
        return (np.floor(u * k) / k).astype(np.float32)
    if kind == "few":
        vals = rng.random(int(rng.integers(1, 6)), dtype=np.float32)
        return vals[rng.integers(0, vals.size, n)]
    if kind == "cluster":
        base = np.float32(rng.random())
        c = np.empty(int(rng.integers(2, 400)), np.float32)
        c[0] = base
        for i in range(1, c.size):
            c[i] = np.nextafter(c[i - 1], np.float32(2))
        s = u.copy()
        m = rng.random(n) < 0.7
        s[m] = c[rng.integers(0, c.size, int(m.sum()))]
        return s
    if kind == "signed":
        s = (np.round((u * 2 - 1) * 50) / 50).astype(np.float32)
        s[rng.random(n) < 0.05] = np.float32(-0.0)
        s[rng.random(n) < 0.05] = np.float32(0.0)
        s[rng.random(n) < 0.001] = np.float32(-3e38)
        s[rng.random(n) < 0.001] = np.float32(3e38)
        return s
    raise ValueError(kind)


def _case(i: int):
    rng = np.random.default_rng(10_000 + i)
    n = int(rng.choice([1_000, 4_097, 65_536, 300_001, 1 << 20, (1 << 21) + 3]))
    kind = ["uniform", "bf16", "grid", "few", "cluster", "signed"][i % 6]
    s = _scores(rng, n, kind)
    p = float(rng.choice([0.0005, 0.01, 0.1, 0.3, 0.5, 0.7]))
    y = np.where(rng.random(n) < p, 1, -1).astype(np.int64)
    if i % 5 == 0:  # labels outside {-1, 1}: negatives, as sklearn's pos_label=1
        y[rng.random(n) < 0.05] = 0
    dtype = [np.int8, np.int32, np.int64][i % 3]
    G = int(rng.integers(2, 9))
    return kind, s, y.astype(dtype), G


def _two_step(ops, ts, ty, G, P, N):
    """ExactAUC's sharded sequence, its G ranks run one after another on one GPU."""
    n = ts.numel()
    nb = ops.auc_slot_bytes(n, G)
    slots = torch.empty(nb * G, dtype=torch.uint8, device=ts.device)
    for r in range(G):
        ops.auc_eval_compact_part(ts, ty, r, G, slots[r * nb:(r + 1) * nb])
    recs = []
    for r in range(G):
        ops.auc_eval_compact_part(ts, ty, r, G, torch.empty(nb, dtype=torch.uint8, device=ts.device))
        recs.append(ops.auc_eval_query_part(ts, ty, r, G, slots).cpu().tolist())
    assert {v[4] for v in recs} == {0}, recs  # the ranks agree
    if any(v[7] == 2 for v in recs):
        if P <= N:
            recs2 = [ops.auc_eval_query_part_sorted(ts, ty, r, G, slots, P).cpu().tolist() for r in range(G)]
            if all(v[7] == 1 for v in recs2):
                return sum(v[0] for v in recs2), sum(v[1] for v in recs2), "sorted_slots"
        W = T = 0
        for r in range(G):
            o = ops.auc_eval_counts_part(ts, ty, r, G, torch.zeros(3, dtype=torch.int64, device=ts.device))
            W, T = W + o[0], T + o[1]
        return W, T, "whole"
    return sum(v[0] for v in recs), sum(v[1] for v in recs), "slotted"


@pytest.mark.parametrize("i", range(N_CASES))
def test_auc_fuzz(dev, i):
    from distributedauc_amd import ops

    kind, s, y, G = _case(i)
    e = coracle.auc_counts(y.astype(np.int64), s)
    ts = torch.from_numpy(s).to(dev)
    ty = torch.from_numpy(y).to(dev)
    W, T, P, N, bad, other = ops.auc_eval_counts(ts, ty)
    assert (W if P and N else 0, T if P and N else 0, P, N, bad) == (
        e["wins"] if e["P"] and e["N"] else 0, e["ties"] if e["P"] and e["N"] else 0, e["P"], e["N"], 0), (i, kind)
    assert other == int(((y != 1) & (y != -1)).sum())
    if e["P"] and e["N"]:
        W2, T2, route = _two_step(ops, ts, ty, G, e["P"], e["N"])
        assert (W2, T2) == (e["wins"], e["ties"]), (i, kind, G, route)


def test_auc_fuzz_nonfinite_raises_in_every_route(dev):
    """A NaN among the negatives of a tie-heavy set (the sorted route) and of a spread one."""
    from distributedauc_amd.auc import ExactAUC

    rng = np.random.default_rng(77)
    for kind in ("uniform", "bf16"):
        s = _scores(rng, 200_001, kind)
        y = np.where(rng.random(s.size) < 0.05, 1, -1).astype(np.int8)
        s[np.flatnonzero(y == -1)[123]] = np.nan
        with pytest.raises(ValueError, match="NaN"):
            ExactAUC().counts(torch.from_numpy(y).to(dev), torch.from_numpy(s).to(dev))
