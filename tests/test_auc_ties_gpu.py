"""The distinct-key index of tie-heavy tables (auc_sort.hip, dk_*_kernel; round 6) vs the C oracle.

The count index refuses a table with a cell of 15+ keys; tie-heavy positive tables (rounded scores,
the probabilities of a bf16 model) are exactly that. The sorted path then counts every query from
the table's DISTINCT keys with the number of table keys <= each, held in LDS (up to 14,000 distinct
keys), instead of the LDS search tree. Every case runs in search mode 0 (the product's choice), 1
(the tree) and 2 (the distinct-key index wherever it holds the table: include/dauc_tuning.h), so
the three structures are checked against each other and against the oracle. Bar: (W, T) bit-exact
against oracle/auc_oracle.c (sklearn's _binary_clf_curve counts, main.py:79-81).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import coracle

pytestmark = pytest.mark.gpu

MODES = (0, 1, 2)


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.fixture
def ops(dev):
    """The tuning build of the library, where the search mode is selectable."""
    from distributedauc_amd import _lib
    from distributedauc_amd import ops as o

    with _lib.using(_lib.tuning()):
        try:
            yield o
        finally:
            o.set_search_mode(0)


def _bf16(a: np.ndarray) -> np.ndarray:
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).bfloat16().float().numpy()


def _oracle_slice(s, y, begin, end):
    pos = s[y == 1]
    neg = s[begin:end][y[begin:end] != 1]
    yy = np.concatenate([np.ones(pos.size, np.int64), -np.ones(neg.size, np.int64)])
    e = coracle.auc_counts(yy, np.concatenate([pos, neg]))
    return e["wins"], e["ties"]


def _check(ops, dev, s, y, begin=0, end=None, what=""):
    end = s.size if end is None else end
    ref = _oracle_slice(s, y, begin, end)
    ts, ty, tpos = T(s, dev), T(y, dev), T(s[y == 1], dev)
    for m in MODES:
        ops.set_search_mode(m)
        wt = torch.zeros(3, dtype=torch.int64, device=dev)
        ops.auc_counts_sorted_labeled(tpos, ts, ty, begin, end, wt, nonfinite=wt[2:])
        got = tuple(wt[:2].cpu().tolist())
        assert got == ref, (what, m, got, ref)
        assert int(wt[2]) == 0, (what, m)


def _labels(rng, n, p, dtype=np.int8):
    return np.where(rng.random(n) < p, 1, -1).astype(dtype)


def _case(name: str, rng, n: int):
    """(scores, labels) of one tie-heavy distribution."""
    y = _labels(rng, n, 0.05)
    u = rng.random(n, dtype=np.float32)
    if name == "bf16":
        s = _bf16(u)
    elif name == "round1e-3":
        s = (np.round(u * 1000) / 1000).astype(np.float32)
    elif name == "sigmoid_bf16_logits":
        z = _bf16(rng.normal(0.0, 2.0, n).astype(np.float32))
        s = (1.0 / (1.0 + np.exp(-z.astype(np.float64)))).astype(np.float32)
    elif name == "all_equal":
        s = u.copy()
        s[y == 1] = np.float32(0.5)
        s[rng.random(n) < 0.01] = np.float32(0.5)  # negatives tied with every positive
    elif name == "two_values":
        s = np.where(u < 0.5, np.float32(0.25), np.float32(0.75)).astype(np.float32)
    elif name == "signed_with_zeros":
        s = (np.round((u * 2 - 1) * 100) / 100).astype(np.float32)
        s[rng.random(n) < 0.05] = np.float32(-0.0)  # -0 ties +0 (fp32 equality)
        s[rng.random(n) < 0.05] = np.float32(0.0)
    elif name == "dense_cluster":
        # 300 consecutive floats (one cell of the plan holds many of them: the binary search),
        # 20 copies each among the positives, plus spread values and queries inside the cluster
        base = np.float32(0.3)
        cluster = np.empty(300, np.float32)
        cluster[0] = base
        for i in range(1, 300):
            cluster[i] = np.nextafter(cluster[i - 1], np.float32(1))
        s = u.copy()
        pi = np.flatnonzero(y == 1)
        s[pi] = cluster[rng.integers(0, 300, pi.size)]
        s[pi[: pi.size // 10]] = _bf16(u[pi[: pi.size // 10]])
        ni = np.flatnonzero(y != 1)
        s[ni[: ni.size // 4]] = cluster[rng.integers(0, 300, ni.size // 4)]
    else:
        raise ValueError(name)
    return s.astype(np.float32), y


CASES = ("bf16", "round1e-3", "sigmoid_bf16_logits", "all_equal", "two_values", "signed_with_zeros", "dense_cluster")


@pytest.mark.parametrize("name", CASES)
def test_distinct_index_tie_heavy(dev, ops, name):
    """Tie-heavy positive tables (the count index refuses them), whole range and a ragged slice
    (scalar head and tail paths), int8 labels."""
    rng = np.random.default_rng(100 + CASES.index(name))
    s, y = _case(name, rng, 1 << 20)
    _check(ops, dev, s, y, what=name)
    _check(ops, dev, s, y, 3, s.size - 5, what=name + " ragged")


@pytest.mark.parametrize("dtype", [np.int32, np.int64])
def test_distinct_index_label_widths(dev, ops, dtype):
    rng = np.random.default_rng(7)
    s, y = _case("bf16", rng, 300_001)
    _check(ops, dev, s, y.astype(dtype), what=str(dtype))
    _check(ops, dev, s, y.astype(dtype), 1, 299_999, what=str(dtype) + " ragged")


@pytest.mark.parametrize("D", [1, 2, 3_200, 3_201, 8192, 13_999, 14_000, 14_001, 20_000])
def test_distinct_index_capacity(dev, ops, D):
    """Exactly D distinct positive values, 16 copies each (a cell of the count index holds 15+:
    refused), queries on, between, below and above them. Up to 14,000 the distinct-key index holds
    the table; past it the tree counts (mode 2 then falls back too)."""
    rng = np.random.default_rng(D)
    vals = np.unique(rng.random(4 * D + 16, dtype=np.float32))[:D]
    assert vals.size == D
    pos = np.repeat(vals, 16)
    neg = np.concatenate([vals[rng.integers(0, D, 50_000)],                      # on the keys
                          rng.random(200_000, dtype=np.float32),                  # between them
                          np.array([-1.0, 0.0, 2.0, vals[0], vals[-1]], np.float32)])  # outside / the ends
    s = np.concatenate([pos, neg]).astype(np.float32)
    y = np.concatenate([np.ones(pos.size, np.int8), -np.ones(neg.size, np.int8)])
    perm = rng.permutation(s.size)
    _check(ops, dev, s[perm], y[perm], what=f"D={D}")


def test_distinct_index_spread_tables_mode2(dev, ops):
    """Mode 2 forces the distinct-key index on tables the count index would hold (few positives,
    no ties): the same counts."""
    rng = np.random.default_rng(11)
    for n, P in ((1 << 18, 1), (1 << 18, 3), (1 << 18, 1000), (1 << 19, 8192)):
        s = rng.random(n, dtype=np.float32)
        y = -np.ones(n, np.int8)
        y[rng.choice(n, P, replace=False)] = 1
        _check(ops, dev, s, y, what=f"P={P}")


@pytest.mark.parametrize("name", ["bf16", "sigmoid_bf16_logits"])
def test_eval_tie_heavy_one_call_and_parts(dev, name):
    """The product library's evaluation on tie-heavy scores (the index refuses the table: verdict 2,
    then the blocking sorted path and its distinct-key index): the one-call counts and the sum of
    4 blocking parts equal the oracle's."""
    from distributedauc_amd import ops as o

    rng = np.random.default_rng(5)
    s, y = _case(name, rng, 1 << 22)
    e = coracle.auc_counts(y.astype(np.int64), s)
    ts, ty = T(s, dev), T(y, dev)
    rec = o.auc_eval_enqueue(ts, ty, 0, 1).cpu().tolist()
    assert rec[7] == 2, rec  # the count index refused the table
    W, Tt, P, N, bad, other = o.auc_eval_counts(ts, ty)
    assert (W, Tt, P, N, bad, other) == (e["wins"], e["ties"], e["P"], e["N"], 0, 0)
    Ws = Ts = 0
    pc = torch.zeros(3, dtype=torch.int64, device=dev)
    for r in range(4):
        w, t, P2, N2, *_ = o.auc_eval_counts_part(ts, ty, r, 4, pc)
        Ws, Ts = Ws + w, Ts + t
        assert (P2, N2) == (e["P"], e["N"])
    assert (Ws, Ts) == (e["wins"], e["ties"])


@pytest.mark.parametrize("p_pos", [0.05, 0.95])
def test_distinct_index_unlabeled_both_table_sides(dev, ops, p_pos):
    """dauc_auc_counts_sorted (materialised classes): the smaller class is the table, the positives
    (p 0.05) or the negatives (p 0.95, W += #(table < x)); bf16-rounded scores, every mode."""
    rng = np.random.default_rng(int(p_pos * 100))
    n = 1 << 20
    s = _bf16(rng.random(n, dtype=np.float32))
    y = _labels(rng, n, p_pos)
    e = coracle.auc_counts(y.astype(np.int64), s)
    pos, neg = T(s[y == 1], dev), T(s[y != 1], dev)
    for m in MODES:
        ops.set_search_mode(m)
        wt = torch.zeros(2, dtype=torch.int64, device=dev)
        ops.auc_counts_sorted(pos, neg, wt)
        assert tuple(wt.cpu().tolist()) == (e["wins"], e["ties"]), (p_pos, m)
        # an unaligned query array (the scalar path of the plain query kernel)
        wt.zero_()
        big = neg if p_pos < 0.5 else pos
        small = pos if p_pos < 0.5 else neg
        tail = big[1:]
        ref = coracle.auc_counts(
            np.concatenate([np.ones(small.numel() if p_pos < 0.5 else tail.numel(), np.int64),
                            -np.ones(tail.numel() if p_pos < 0.5 else small.numel(), np.int64)]),
            np.concatenate([small.cpu().numpy(), tail.cpu().numpy()] if p_pos < 0.5
                           else [tail.cpu().numpy(), small.cpu().numpy()]))
        if p_pos < 0.5:
            ops.auc_counts_sorted(small, tail, wt)
        else:
            ops.auc_counts_sorted(tail, small, wt)
        assert tuple(wt.cpu().tolist()) == (ref["wins"], ref["ties"]), (p_pos, m, "unaligned")


def test_eval_tie_heavy_positive_majority(dev):
    """The product evaluation when the negatives are the smaller class of a tie-heavy test set:
    verdict 2, the split and the distinct-key index over the negatives; the oracle's counts."""
    from distributedauc_amd import ops as o

    rng = np.random.default_rng(9)
    n = 1 << 21
    s = _bf16(rng.random(n, dtype=np.float32))
    y = _labels(rng, n, 0.9)
    e = coracle.auc_counts(y.astype(np.int64), s)
    W, Tt, P, N, bad, other = o.auc_eval_counts(T(s, dev), T(y, dev))
    assert (W, Tt, P, N, bad, other) == (e["wins"], e["ties"], e["P"], e["N"], 0, 0)
