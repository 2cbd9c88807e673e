"""Pin the CPU oracle to the reference's own outputs (tests/golden/, made by make_golden.py).

The oracle is only trusted as a checker after it reproduces every golden vector.
"""
from __future__ import annotations

import hashlib
import json

import numpy as np
import pytest
import torch

from oracle import coracle
from oracle import reference_cpu as R


def test_surrogate_fp32_bitwise(golden):
    z = np.load(golden / "surrogate_cases.npz")
    for ci in range(int(z["ncases"])):
        h, y, abap = z[f"c{ci}_h"], z[f"c{ci}_y"].astype(np.int64), z[f"c{ci}_abap"]
        F, dh, da, db, dal = R.surrogate_fwdbwd_fp32(h, y, *abap)
        assert np.array_equal(np.array([F, da, db, dal], np.float32), z[f"c{ci}_fp32"]), ci
        assert np.array_equal(dh, z[f"c{ci}_dh32"]), ci


def test_surrogate_closed_form_vs_autograd(golden):
    """fp64 closed form (the kernels' formula) vs the reference's fp32 autograd: 1e-5 of the term scale."""
    z = np.load(golden / "surrogate_cases.npz")
    for ci in range(int(z["ncases"])):
        h, y, abap = z[f"c{ci}_h"], z[f"c{ci}_y"].astype(np.int64), z[f"c{ci}_abap"]
        F, dh, da, db, dal = R.surrogate_closed_form(h, y, *abap)
        ref = z[f"c{ci}_fp32"].astype(np.float64)
        scale = np.abs(ref) + 2.0 * np.abs(1 + abap[2]) * np.mean(h) + 1e-3
        assert np.all(np.abs(np.array([F, da, db, dal]) - ref) <= 1e-5 * scale), ci
        assert np.allclose(z[f"c{ci}_fp64"], [F, da, db, dal], rtol=0, atol=0)


def test_dppd_sg_bitwise(golden):
    z = np.load(golden / "dppd_sg.npz")
    lr, gamma = float(z["lr"]), float(z["gamma"])
    assert np.array_equal(R.dppd_sg_flat(z["w"], z["g"], z["w0"], lr, gamma), z["w_new"])
    assert np.array_equal(coracle.pd_update(z["w"], z["g"], z["w0"], lr, gamma), z["w_new"])
    s, g, an = z["scalars"], z["grad3"], z["anchor3"]
    got = R.scalar_update(*s, *g, *an, lr, gamma, "reference")
    assert np.array_equal(np.array(got, np.float32), z["scalars_new"])


def test_auc_counts_and_float(golden):
    z = np.load(golden / "auc_cases.npz")
    for name in z["names"]:
        y, s = z[f"{name}_y"], z[f"{name}_s"]
        W, T, P, N, two_u = (int(v) for v in z[f"{name}_counts"])
        c = coracle.auc_counts(y, s)
        assert (c["wins"], c["ties"], c["P"], c["N"]) == (W, T, P, N), name
        p = R.auc_counts(y, s)
        assert p["two_u"] == two_u == 2 * W + T, name
        ref = float(z[f"{name}_auc"])
        assert abs(R.auc_from_counts(W, T, P, N) - ref) <= 4 * np.spacing(ref), name
        assert R.auc_sklearn(y, s) == ref, name


def test_auc_nonfinite_raises():
    with pytest.raises(ValueError):
        coracle.auc_counts([1, -1], [np.nan, 0.5])
    with pytest.raises(ValueError):
        R.auc_counts([1, -1], [np.inf, 0.5])


def test_pair_count_bruteforce_matches_sort(golden):
    z = np.load(golden / "auc_cases.npz")
    for name in ("ties_1k", "signed_zero", "subnormal", "all_equal"):
        y, s = z[f"{name}_y"], z[f"{name}_s"]
        W, T, *_ = (int(v) for v in z[f"{name}_counts"])
        assert coracle.pair_count_bruteforce(s[y == 1], s[y != 1]) == (W, T), name


def test_partition_indices(golden):
    ref = json.loads((golden / "partitions.json").read_text())
    for keep in (0.4, 1.0):
        for size in (1, 4):  # the rest are covered by tests/test_host.py through the product partitioner
            parts = R.partition_indices([0.01] + [(1 - 0.01) / size] * size, 123, keep)
            for p, r in zip(parts, ref[f"keep{keep}_size{size}"]):
                assert len(p) == r["len"]
                assert hashlib.sha256(np.asarray(p, np.int64).tobytes()).hexdigest() == r["sha256"]


def test_label_map_phat_match_coda_trajectory(golden):
    """p_hat recorded by the reference at every step equals the restated formula on its counts."""
    z = np.load(golden / "coda_w2.npz")
    for r in (0, 1):
        for (gp, gn, lp, ln), ph in zip(z[f"r{r}_counts"], z[f"r{r}_p_hat"]):
            assert R.phat(gp, gn, lp, ln) == np.float32(ph)


def test_coda_average_restatement(golden):
    z = np.load(golden / "coda_w2.npz")
    a, b = np.float32([1.5, -2.25, 3.0]), np.float32([0.5, 0.25, -1.0])
    assert np.array_equal(R.coda_average([a, b]), (torch.tensor(a) + torch.tensor(b)).div(2.0).numpy())
    assert z["world"] == 2
