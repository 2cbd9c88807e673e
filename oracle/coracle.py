"""ctypes binding of oracle/build/liboracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; never by the product package.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "liboracle.so"
_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists() or LIB.stat().st_mtime < (HERE / "auc_oracle.c").stat().st_mtime:
            build()
        L = ctypes.CDLL(str(LIB))
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.oracle_auc_counts.argtypes = [vp, vp, i64, vp]
        L.oracle_auc_counts.restype = ctypes.c_int
        L.oracle_pair_count_bruteforce.argtypes = [vp, i64, vp, i64, vp]
        L.oracle_pair_count_bruteforce.restype = None
        L.oracle_pd_update.argtypes = [vp, vp, vp, vp, i64, ctypes.c_float, ctypes.c_float]
        L.oracle_pd_update.restype = None
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def auc_counts(labels, scores) -> dict:
    """Exact (W, T, P, N) of sklearn's ROC area; ValueError on non-finite scores."""
    s = np.ascontiguousarray(scores, dtype=np.float32).reshape(-1)
    y = np.ascontiguousarray(labels, dtype=np.int64).reshape(-1)
    out = np.zeros(4, np.uint64)
    rc = lib().oracle_auc_counts(_p(s), _p(y), s.size, _p(out))
    if rc == -1:
        raise ValueError("Input contains NaN or infinity.")
    if rc != 0:
        raise MemoryError("oracle_auc_counts failed")
    return {"wins": int(out[0]), "ties": int(out[1]), "P": int(out[2]), "N": int(out[3])}


def pair_count_bruteforce(pos, neg) -> tuple[int, int]:
    p = np.ascontiguousarray(pos, np.float32)
    n = np.ascontiguousarray(neg, np.float32)
    out = np.zeros(2, np.uint64)
    lib().oracle_pair_count_bruteforce(_p(p), p.size, _p(n), n.size, _p(out))
    return int(out[0]), int(out[1])


def pd_update(w, g, w0, lr, gamma, avg=None):
    """fp32 main.py:61 (+ 333-334 when avg is given); returns new copies."""
    w = np.array(w, np.float32, copy=True)
    g = np.ascontiguousarray(g, np.float32)
    w0 = np.ascontiguousarray(w0, np.float32)
    a = None if avg is None else np.array(avg, np.float32, copy=True)
    lib().oracle_pd_update(_p(w), _p(g), _p(w0), None if a is None else _p(a), w.size,
                           np.float32(lr), np.float32(1 / gamma))
    return w if a is None else (w, a)
