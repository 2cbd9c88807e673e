"""The search structures of the sort method (auc_sort.hip; dauc_set_search_mode of the tuning build,
include/dauc_tuning.h) vs the C oracle.

The labeled query pass (dauc_auc_counts_sorted_labeled, and through it dauc_auc_eval_counts)
locates every negative among the sorted positives through one of: the count index (mode 0, the
default where it fits: top 11 key bits -> bucket, multiply-high -> cell, per-8-cell LDS words of
base + nibble counts, one 16-byte window for non-empty cells; the device falls back to the tree
for skewed tables) or the LDS search tree (mode 1). Every case here runs in both modes, so the
skewed cases also cover mode 0's device-side fallback. (Round 2's 16-key-slot cell index, a
measured and slower alternative, was removed in round 4.) Bar: the integers (W, T) bit-exact against oracle/auc_oracle.c (sklearn's
_binary_clf_curve counts, main.py:79-81) on the same scores.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import coracle

pytestmark = pytest.mark.gpu

MODES = (0, 1)


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.fixture
def ops(dev):
    """The ops run against the tuning build of the library, where the search mode is selectable."""
    from distributedauc_amd import _lib
    from distributedauc_amd import ops as o

    with _lib.using(_lib.tuning()):
        try:
            yield o
        finally:
            o.set_search_mode(0)
            o.set_direct_fault(0)
            o.set_index_form(0)


def _oracle_slice(s, y, begin, end):
    """(W, T) of all positives against the slice's non-positives (labels != 1)."""
    pos = s[y == 1]
    neg = s[begin:end][y[begin:end] != 1]
    yy = np.concatenate([np.ones(pos.size, np.int64), -np.ones(neg.size, np.int64)])
    e = coracle.auc_counts(yy, np.concatenate([pos, neg]))
    return e["wins"], e["ties"]


def _check(ops, dev, s, y, begin=0, end=None, modes=MODES, what=""):
    end = s.size if end is None else end
    ref = _oracle_slice(s, y, begin, end)
    ts, ty = T(s, dev), T(y, dev)
    tpos = T(s[y == 1], dev)
    for m in modes:
        ops.set_search_mode(m)
        wt = torch.zeros(3, dtype=torch.int64, device=dev)
        ops.auc_counts_sorted_labeled(tpos, ts, ty, begin, end, wt, nonfinite=wt[2:])
        got = tuple(wt[:2].cpu().tolist())
        assert got == ref, (what, m, got, ref)
        assert int(wt[2]) == 0, (what, m)


def _labels(rng, n, p, dtype=np.int8):
    return np.where(rng.random(n) < p, 1, -1).astype(dtype)


def test_cells_uniform_scores(dev, ops):
    """The bench's distribution (U(0,1) fp32, loader.synthetic_scores) at table sizes that need
    mu = 4, 5 and 6 keys per cell (134k, 168k, 200k positives) and a few small tables."""
    rng = np.random.default_rng(1)
    for n, P in ((1 << 20, 1), (1 << 20, 2), (1 << 20, 17), (1 << 20, 4_000), (1 << 21, 134_447),
                 (1 << 21, 168_478), (1 << 21, 200_000)):
        s = rng.random(n, dtype=np.float32)
        y = -np.ones(n, np.int8)
        y[rng.choice(n, P, replace=False)] = 1
        _check(ops, dev, s, y, what=(n, P))


def test_cells_signed_wide_and_special_values(dev, ops):
    """Normal scores of both signs over 60 binades, +-0, subnormals, the largest finite values:
    keys spread over many top buckets, empty buckets between them, ties between -0 and +0."""
    rng = np.random.default_rng(2)
    n = 1 << 20
    s = (rng.standard_normal(n) * np.exp2(rng.integers(-30, 30, n))).astype(np.float32)
    special = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-40, -1e-40, 3.4e38, -3.4e38, 1.0, -1.0], np.float32)
    k = rng.random(n) < 0.02
    s[k] = rng.choice(special, int(k.sum()))
    y = _labels(rng, n, 0.03)
    _check(ops, dev, s, y, what="wide")
    # all positives at the two extremes of the key range (first and last top buckets)
    s2 = rng.random(n, dtype=np.float32) - 0.5
    y2 = _labels(rng, n, 0.0)
    y2[:50] = 1
    s2[:25] = -3.4e38
    s2[25:50] = 3.4e38
    _check(ops, dev, s2, y2, what="extremes")


def test_cells_ties_and_overflowing_cells(dev, ops):
    """Quantised scores: runs of equal keys longer than a 16-key slot (the slot-cell pass
    searches the rest of the cell in global memory; the count index finds a cell of 15+ keys
    and keeps the tree), and a run of 20 equal keys in one cell with the rest of the table
    uniform, ties across cell edges."""
    rng = np.random.default_rng(3)
    n = 1 << 20
    for levels, p in ((3001, 0.01), (97, 0.05), (5, 0.2), (1, 0.01)):
        s = (np.floor(rng.random(n) * levels) / levels).astype(np.float32)
        y = _labels(rng, n, p)
        _check(ops, dev, s, y, what=("levels", levels))
    s = rng.random(n, dtype=np.float32)
    y = _labels(rng, n, 0.02)
    pos_idx = np.flatnonzero(y == 1)
    s[pos_idx[:20]] = np.float32(0.625)        # one cell holds a 20-key run of 0.625
    neg_idx = np.flatnonzero(y == -1)
    s[neg_idx[:1000]] = np.float32(0.625)      # negatives tied with it
    s[neg_idx[1000:2000]] = np.nextafter(np.float32(0.625), np.float32(1))
    s[neg_idx[2000:3000]] = np.nextafter(np.float32(0.625), np.float32(0))
    _check(ops, dev, s, y, what="run of 20")


def test_cells_clustered_table(dev, ops):
    """90 % of the positives inside a 1e-4-wide interval: the cells of their top bucket hold
    hundreds of keys each (slot + binary search in the cell pass)."""
    rng = np.random.default_rng(4)
    n = 1 << 20
    s = rng.random(n, dtype=np.float32)
    y = _labels(rng, n, 0.01)
    pos_idx = np.flatnonzero(y == 1)
    c = pos_idx[: int(0.9 * pos_idx.size)]
    s[c] = (0.7 + 1e-4 * rng.random(c.size)).astype(np.float32)
    neg_idx = np.flatnonzero(y == -1)
    s[neg_idx[:50_000]] = (0.7 + 1e-4 * rng.random(50_000)).astype(np.float32)
    _check(ops, dev, s, y, what="cluster")


@pytest.mark.parametrize("ldtype", [np.int8, np.int32, np.int64])
def test_cells_label_types_and_ranges(dev, ops, ldtype):
    """Unaligned [begin, end) slices (the sharded evaluation's index ranges), labels 0 (a
    negative for pos_label=1), every label dtype."""
    rng = np.random.default_rng(5)
    n = 300_001
    s = rng.random(n, dtype=np.float32)
    y = _labels(rng, n, 0.02, ldtype)
    y[rng.random(n) < 0.01] = 0
    for begin, end in ((0, n), (3, n - 5), (1, 2), (n // 3, 2 * n // 3 + 1), (7, 7)):
        _check(ops, dev, s, y, begin, end, what=(begin, end))


def test_cells_table_size_limits(dev, ops):
    """Table sizes around the limits: the count index up to 1.5 keys per cell (215,040 uses it,
    400,000 is past it: the tree), the slot-cell index up to 16 keys per cell (573,440) and one
    key past it (the tree in every mode)."""
    rng = np.random.default_rng(6)
    n = 1 << 22
    for P in (215_040, 215_041, 400_000, 573_440, 573_441):
        s = rng.random(n, dtype=np.float32)
        y = -np.ones(n, np.int8)
        y[rng.choice(n, P, replace=False)] = 1
        _check(ops, dev, s, y, what=P)


def test_cells_one_call_eval(dev, ops):
    """dauc_auc_eval_counts in every mode, the speculative table size included (the same data
    twice, then other data of the same length)."""
    rng = np.random.default_rng(7)
    n = 1 << 21
    data = [(rng.random(n, dtype=np.float32), _labels(rng, n, p)) for p in (0.001, 0.01, 0.001)]
    for m in MODES:
        ops.set_search_mode(m)
        for s, y in (data[0], data[0], data[1], data[2], data[2]):
            W, Tt, P, N, bad, other = ops.auc_eval_counts(T(s, dev), T(y, dev))
            e = coracle.auc_counts(y.astype(np.int64), s)
            assert (W, Tt, P, N, bad) == (e["wins"], e["ties"], e["P"], e["N"], 0), m


def test_cells_rejects_nonfinite_queries(dev, ops):
    """A NaN / inf negative is counted by the cell pass too (sklearn _ranking.py:868-869)."""
    rng = np.random.default_rng(8)
    n = 100_003
    for m in MODES:
        ops.set_search_mode(m)
        for bad in (np.nan, np.inf, -np.inf):
            s = rng.random(n, dtype=np.float32)
            y = _labels(rng, n, 0.01)
            s[int(np.flatnonzero(y == -1)[5])] = bad
            wt = torch.zeros(3, dtype=torch.int64, device=dev)
            ops.auc_counts_sorted_labeled(T(s[y == 1], dev), T(s, dev), T(y, dev), 0, n, wt, nonfinite=wt[2:])
            assert int(wt[2]) == 1, (m, bad)


def test_search_mode_rejects_unknown(dev, ops):
    from distributedauc_amd._lib import DaucError

    with pytest.raises(DaucError):
        ops.set_search_mode(3)


@pytest.mark.parametrize("fault", [1, 2, 3])
def test_direct_build_guards_bad_indices(dev, ops, fault):
    """The direct count-index build checks every cell index and counter before its scatter stores
    (auc_sort.hip, direct_scatter_kernel): the tuning build corrupts one key's cell (past the last
    cell / moved to the next cell) or one cell's counter between the count and scatter passes, and
    the evaluation reports verdict 2 -- the blocking call then takes the sorted path and returns
    the oracle's exact counts. Without the fault the same data is counted by the index (verdict 1)."""
    ops.set_index_form(1)  # round 5's direct build (the slotted build has no scatter to guard)
    rng = np.random.default_rng(9 + fault)
    n = 1 << 21
    data = [(rng.random(n, dtype=np.float32), _labels(rng, n, p)) for p in (0.01, 0.001)]
    for s, y in data:
        e = coracle.auc_counts(y.astype(np.int64), s)
        ts, ty = T(s, dev), T(y, dev)
        ops.set_direct_fault(0)
        rec = ops.auc_eval_enqueue(ts, ty, 0, 1).cpu().tolist()
        assert rec[7] == 1 and tuple(rec[:2]) == (e["wins"], e["ties"]), rec
        ops.set_direct_fault(fault)
        rec = ops.auc_eval_enqueue(ts, ty, 0, 1).cpu().tolist()
        assert rec[7] == 2, (fault, rec)
        W, Tt, P, N, bad, other = ops.auc_eval_counts(ts, ty)
        assert (W, Tt, P, N, bad, other) == (e["wins"], e["ties"], e["P"], e["N"], 0, 0), fault
        ops.set_direct_fault(0)
        W, Tt, P, N, bad, other = ops.auc_eval_counts(ts, ty)
        assert (W, Tt, P, N) == (e["wins"], e["ties"], e["P"], e["N"])


@pytest.mark.parametrize("case", ["uniform", "ties", "cells_5_14", "cell_15", "p_over_half"])
def test_index_forms_agree_one_call(dev, ops, case):
    """The one-call evaluation (dauc_auc_eval_enqueue / _counts) with the count index built by round 5's
    direct build (form 1: count, blocks, scatter) and by round 6's slotted build (form 0, the
    product's): the same record, word for word, and the C oracle's counts. Cases: uniform scores;
    tie-heavy quantised scores; positives repeated 5..14 times in one cell (the secondary window and
    the tertiary run); a cell of 15 (both forms refuse the index: verdict 2, then the sorted path);
    more positives than negatives."""
    rng = np.random.default_rng({"uniform": 1, "ties": 2, "cells_5_14": 3, "cell_15": 4, "p_over_half": 5}[case])
    n = 1_000_003
    s = rng.random(n, dtype=np.float32)
    p = 0.6 if case == "p_over_half" else 0.02
    y = np.where(rng.random(n) < p, 1, -1).astype(np.int8)
    if case == "ties":
        s = (np.floor(s * 20000) / 20000).astype(np.float32)
    if case in ("cells_5_14", "cell_15"):
        s = (s * np.float32(0.25)).astype(np.float32)
        pos, neg = np.flatnonzero(y == 1), np.flatnonzero(y == -1)
        at = 0
        for j, m in enumerate((5, 8, 9, 14) if case == "cells_5_14" else (15,)):
            v = np.float32(0.3 + 0.1 * j)
            s[pos[at:at + m]] = v
            at += m
            s[neg[50 * j:50 * j + 9]] = v
            s[neg[50 * j + 9:50 * j + 12]] = np.nextafter(v, np.float32(1))
    e = coracle.auc_counts(y.astype(np.int64), s)
    ts, ty = T(s, dev), T(y, dev)
    recs = {}
    for form in (1, 0):
        ops.set_index_form(form)
        recs[form] = ops.auc_eval_enqueue(ts, ty, 0, 1).cpu().tolist()
        W, Tt, P, N, bad, other = ops.auc_eval_counts(ts, ty)
        assert (W, Tt, P, N, bad) == (e["wins"], e["ties"], e["P"], e["N"], 0), (case, form)
    assert recs[0] == recs[1], (case, recs)
    want = 2 if case in ("cell_15", "p_over_half") else 1
    assert recs[0][7] == want, (case, recs[0])
