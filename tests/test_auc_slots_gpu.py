"""The range-slot query path of the one-call evaluation (tuning_slots.hip; dauc_set_query_path(2) of
the tuning build, include/dauc_tuning.h) against the C oracle and the count-index path.

The evaluation compacts the positives, builds the range-slot index straight from them (cells of
the count index's map at ~2 cells per key, ranges of 8192 cells, a 16-byte slot per cell), splits
the queries by range and counts each range from its slots in LDS. Bar: the integers (W, T, P, N,
non-finite, other labels) bit-exact against oracle/auc_oracle.c (sklearn's _binary_clf_curve
counts, main.py:79-81) on the same scores, and the parts of a sharded evaluation summing to the
whole. Tables the index cannot hold (a cell of 16+ keys, more than 1.5 keys per cell) report
verdict 2 and the blocking call's sorted path returns the same integers.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import coracle

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.fixture
def ops(dev):
    """The ops run against the tuning build of the library with the range-slot query path."""
    from distributedauc_amd import _lib
    from distributedauc_amd import ops as o

    with _lib.using(_lib.tuning()):
        o.set_query_path(2)
        try:
            yield o
        finally:
            o.set_query_path(1)


def _labels(rng, n, p, dtype=np.int8):
    return np.where(rng.random(n) < p, 1, -1).astype(dtype)


def _check(ops, dev, s, y, verdict=1, parts=(1,), what=""):
    """verdict: the one every non-empty part must report (None: either; ties decide)."""
    e = coracle.auc_counts(y.astype(np.int64), s)
    ts, ty = T(s, dev), T(y, dev)
    W, Tt, P, N, bad, other = ops.auc_eval_counts(ts, ty)
    assert (W, Tt, P, N, bad, other) == (e["wins"], e["ties"], e["P"], e["N"], 0, 0), (what, W, Tt, e)
    for G in parts:
        recs = [ops.auc_eval_enqueue(ts, ty, r, G).cpu().tolist() for r in range(G)]
        got_v = {r[7] for r in recs if r[7] != 0}
        assert verdict is None or got_v <= {verdict}, (what, G, got_v)
        if got_v == {1}:
            assert (sum(r[0] for r in recs), sum(r[1] for r in recs)) == (e["wins"], e["ties"]), (what, G)
            assert all(r[3] == e["P"] for r in recs)


def test_slots_uniform_scores(dev, ops):
    """The bench's distribution at table sizes from 1 key to past round 3's count-index limit
    (219,838 keys): 838 k positives take ~1 M cells (0.8 keys per cell)."""
    rng = np.random.default_rng(1)
    for n, P in ((1 << 20, 1), (1 << 20, 3), (1 << 20, 4_000), (1 << 21, 134_447), (1 << 21, 200_000),
                 (1 << 22, 838_861)):
        s = rng.random(n, dtype=np.float32)
        y = -np.ones(n, np.int8)
        y[rng.choice(n, P, replace=False)] = 1
        _check(ops, dev, s, y, parts=(1, 3) if P > 3 else (1,), what=(n, P))


def test_slots_configs4_size(dev, ops):
    """configs[4]: 2^27 scores at 0.1 % positives, bit-exact, whole and in 8 parts."""
    from distributedauc_amd.loader import synthetic_scores

    s, y = synthetic_scores(1 << 27, 0.001, dev)
    sn, yn = s.cpu().numpy(), y.cpu().numpy()
    _check(ops, dev, sn, yn, parts=(8,), what="configs4")


def test_slots_wide_and_special_values(dev, ops):
    """Normal scores of both signs over 60 binades, +-0, subnormals, the largest finite values:
    ranges spanning many small top buckets, empty buckets between used ones, queries in empty
    buckets and above the last cell."""
    rng = np.random.default_rng(2)
    n = 1 << 20
    s = (rng.standard_normal(n) * np.exp2(rng.integers(-30, 30, n))).astype(np.float32)
    special = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-40, -1e-40, 3.4e38, -3.4e38, 1.0, -1.0], np.float32)
    k = rng.random(n) < 0.02
    s[k] = rng.choice(special, int(k.sum()))
    y = _labels(rng, n, 0.03)
    # ~600 positives tied at each special value: cells of 16+ keys (verdict 2) are likely
    _check(ops, dev, s, y, verdict=None, parts=(1, 4), what="wide")
    s2 = rng.random(n, dtype=np.float32) - 0.5
    y2 = _labels(rng, n, 0.0)
    y2[:50] = 1
    s2[:25] = -3.4e38
    s2[25:50] = 3.4e38
    _check(ops, dev, s2, y2, verdict=2, what="extremes")  # 25 tied positives at each extreme: one cell
    # positives only in the middle: queries below the first and above the last used bucket
    s3 = rng.random(n, dtype=np.float32) * 4.0 - 2.0
    y3 = np.where((np.abs(s3) < 0.25) & (rng.random(n) < 0.3), 1, -1).astype(np.int8)
    _check(ops, dev, s3, y3, parts=(1, 2), what="middle")


def test_slots_ties_and_skew(dev, ops):
    """Quantised scores: runs of equal keys in one cell (4..15 keys read past the slot from the
    table; 16+ keys make the table unusable: verdict 2 and the sorted path), a run of 12 equal
    positives with the rest uniform, ties across cell edges."""
    rng = np.random.default_rng(3)
    n = 1 << 20
    s = (np.floor(rng.random(n) * 100_003) / 100_003).astype(np.float32)
    y = _labels(rng, n, 0.01)
    _check(ops, dev, s, y, parts=(1, 2), what="100k levels")
    for levels, p in ((97, 0.05), (1, 0.01)):
        s = (np.floor(rng.random(n) * levels) / levels).astype(np.float32)
        y = _labels(rng, n, p)
        _check(ops, dev, s, y, verdict=2, parts=(1, 2), what=("levels", levels))
    s = rng.random(n, dtype=np.float32)
    y = _labels(rng, n, 0.02)
    pos_idx = np.flatnonzero(y == 1)
    s[pos_idx[:12]] = np.float32(0.625)
    neg_idx = np.flatnonzero(y == -1)
    s[neg_idx[:1000]] = np.float32(0.625)
    s[neg_idx[1000:2000]] = np.nextafter(np.float32(0.625), np.float32(1))
    s[neg_idx[2000:3000]] = np.nextafter(np.float32(0.625), np.float32(0))
    _check(ops, dev, s, y, parts=(1, 2), what="run of 12")


@pytest.mark.parametrize("ldtype", [np.int8, np.int32, np.int64])
def test_slots_label_types_and_parts(dev, ops, ldtype):
    """Every label dtype, labels 0 (negatives for pos_label=1), lengths that are not multiples of
    4 or of a split tile, sharded parts with unaligned boundaries (G = 1..5, 8)."""
    rng = np.random.default_rng(5)
    for n in (1, 7, 1000, 300_001, 1 << 20):
        s = rng.random(n, dtype=np.float32)
        y = _labels(rng, n, 0.02, ldtype)
        y[rng.random(n) < 0.01] = 0
        if n == 1:
            y[:] = -1
        e = coracle.auc_counts(np.where(y == 1, 1, -1).astype(np.int64), s)
        ts, ty = T(s, dev), T(y, dev)
        W, Tt, P, N, bad, other = ops.auc_eval_counts(ts, ty)
        assert (W, Tt, P, N, bad) == (e["wins"], e["ties"], e["P"], e["N"], 0), n
        assert other == int((y == 0).sum())
        if e["P"] == 0 or e["N"] == 0:
            continue
        for G in (2, 3, 5, 8):
            recs = [ops.auc_eval_enqueue(ts, ty, r, G).cpu().tolist() for r in range(G)]
            assert all(r[7] in (0, 1) for r in recs), (n, G)
            assert (sum(r[0] for r in recs), sum(r[1] for r in recs)) == (e["wins"], e["ties"]), (n, G)


def test_slots_nonfinite(dev, ops):
    """A NaN / inf negative is counted by the split (sklearn _ranking.py:868-869), also when the
    table is empty (no positives: the split only checks finiteness)."""
    rng = np.random.default_rng(8)
    n = 100_003
    for bad in (np.nan, np.inf, -np.inf):
        s = rng.random(n, dtype=np.float32)
        y = _labels(rng, n, 0.01)
        s[int(np.flatnonzero(y == -1)[5])] = bad
        rec = ops.auc_eval_enqueue(T(s, dev), T(y, dev), 0, 1).cpu().tolist()
        assert rec[2] == 1, (bad, rec)
        y0 = -np.ones(n, np.int8)
        rec = ops.auc_eval_enqueue(T(s, dev), T(y0, dev), 0, 1).cpu().tolist()
        assert rec[2] == 1 and rec[3] == 0, (bad, rec)


def test_slots_two_step_parts(dev, ops):
    """The two-step sharded form (compact part -> gathered slots -> query part) on the slot path."""
    rng = np.random.default_rng(9)
    n = 1 << 21
    s = rng.random(n, dtype=np.float32)
    y = _labels(rng, n, 0.01)
    e = coracle.auc_counts(y.astype(np.int64), s)
    ts, ty = T(s, dev), T(y, dev)
    for G in (1, 2, 8):
        nb = ops.auc_slot_bytes(n, G)
        slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
        for r in range(G):
            ops.auc_eval_compact_part(ts, ty, r, G, slots[r * nb:(r + 1) * nb])
        recs = [ops.auc_eval_query_part(ts, ty, r, G, slots).cpu().tolist() for r in range(G)]
        assert all(r[7] == 1 for r in recs), G
        assert (sum(r[0] for r in recs), sum(r[1] for r in recs)) == (e["wins"], e["ties"]), G
