"""Micro-benchmarks of the hot kernels (HIP events on the launch stream), one process.

  update     dauc_pd_update_dense, n = 23,512,130 (ResNet-50), 24 B/param, every variant
  copy       torch D2D copy of 1 GiB: the practical HBM ceiling next to the 8 TB/s spec
  surrogate  dauc_surrogate_fwdbwd at B = 2^26 (9 B/element) and B = 256 (latency)
  paircount  dauc_pair_count_variant at 2^24 scores, 1 % positives, every variant (counts must agree)

Prints one JSON object per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributedauc_amd import _lib, ops  # noqa: E402


def timeit(fn, reps, warm=3):
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        ts.append((a, b))
    torch.cuda.synchronize()
    v = [a.elapsed_time(b) for a, b in ts]
    return float(np.median(v)), float(np.min(v))


def emit(**kw):
    print(json.dumps(kw), flush=True)


def bench_update(dev, reps, variants=range(8)):
    n = 23_512_130
    g = torch.Generator(device=dev).manual_seed(0)
    base = [torch.randn(n, device=dev, generator=g) for _ in range(4)]
    ref = None
    for v in variants:
        w, gr, w0, avg = (t.clone() for t in base)
        ops.pd_update_dense(w, gr, w0, avg, lr=0.1, gamma=2000.0, variant=v)
        if ref is None:
            ref = (w.clone(), avg.clone())
        same = bool(torch.equal(ref[0], w) and torch.equal(ref[1], avg))
        med, mn = timeit(lambda: ops.pd_update_dense(w, gr, w0, avg, lr=0.1, gamma=2000.0, variant=v), reps)
        emit(kernel="pd_update", variant=v, n=n, us=med * 1e3, us_min=mn * 1e3, GBps=24 * n / med / 1e6,
             GBps_best=24 * n / mn / 1e6, bitexact_vs_v0=same)
    for v in list(variants)[:1]:
        w, gr, w0 = (t.clone() for t in base[:3])
        med, mn = timeit(lambda: ops.pd_update_dense(w, gr, w0, None, lr=0.1, gamma=2000.0, variant=v), reps)
        emit(kernel="pd_update_noavg", variant=v, n=n, us=med * 1e3, GBps=16 * n / med / 1e6)


def bench_copy(dev, reps):
    n = 1 << 28  # 1 GiB of fp32
    a = torch.empty(n, device=dev).normal_()
    b = torch.empty_like(a)
    med, mn = timeit(lambda: b.copy_(a), reps)
    emit(kernel="torch_copy_1GiB", us=med * 1e3, GBps=8 * n / med / 1e6, GBps_best=8 * n / mn / 1e6)
    n2 = 23_512_130 * 3  # update-sized working set
    a2, b2 = a[:n2], b[:n2]
    med, mn = timeit(lambda: b2.copy_(a2), reps)
    emit(kernel="torch_copy_282MB", us=med * 1e3, GBps=8 * n2 / med / 1e6)


def bench_surrogate(dev, reps, variants=(0,)):
    """variant 0 = default dispatch; 1 = persistent grid-stride kernel; 2..7 = chunk geometries."""
    for B in (1 << 26, 1 << 24, 1 << 22, 1 << 20, 256):
        g = torch.Generator(device=dev).manual_seed(1)
        h = torch.rand(B, device=dev, generator=g)
        y = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
        ab = torch.tensor([0.1, -0.2, 0.3], device=dev)
        p = torch.tensor([0.1], device=dev)
        dh = torch.empty(B, device=dev)
        g3 = torch.empty(3, device=dev)
        ref = None
        if B >= (1 << 24):
            # practical ceilings for this access mix: torch's own streaming kernels
            med, _ = timeit(lambda: dh.copy_(h), reps)
            emit(kernel="ceiling_copy_f32", B=B, us=med * 1e3, GBps=8 * B / med / 1e6)
            med, _ = timeit(lambda: torch.mul(h, y, out=dh), reps)
            emit(kernel="ceiling_mul_f32_i8", B=B, us=med * 1e3, GBps=9 * B / med / 1e6)
        for v in (variants if B >= 4096 else (0,)):
            ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, grad3=g3, variant=v)
            got = dh.clone()
            ref = got if ref is None else ref
            med, mn = timeit(lambda: ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, grad3=g3, variant=v), reps)
            emit(kernel="surrogate", variant=v, B=B, us=med * 1e3, us_min=mn * 1e3, GBps=9 * B / med / 1e6,
                 GBps_best=9 * B / mn / 1e6, dh_equal_v0=bool(torch.equal(got, ref)))


def timeit_b2b(fn, reps, warm=3):
    """One event pair around reps back-to-back calls (no per-call marker packets): ms per call."""
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps


def bench_surrogate_b2b(dev, reps, variants):
    """B = 2^26: each variant timed over reps back-to-back calls (what the bench line reports)."""
    B = 1 << 26
    g = torch.Generator(device=dev).manual_seed(7)
    h = torch.rand(B, device=dev, generator=g)
    y = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
    ab = torch.tensor([0.1, -0.2, 0.3], device=dev)
    p = torch.tensor([0.1], device=dev)
    dh = torch.empty(B, device=dev)
    g3 = torch.empty(3, device=dev)
    o = torch.zeros(6, dtype=torch.float64, device=dev)
    for v in variants:
        ms = timeit_b2b(lambda: ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, grad3=g3, out64=o, variant=v), reps)
        emit(kernel="surrogate_b2b", variant=v, B=B, us=ms * 1e3, GBps=9 * B / ms / 1e6, frac=9 * B / ms / 1e6 / 8000)


def bench_aucsort(dev, reps):
    """The sort-method evaluation by stage: compaction (labels + positives' scores), the
    whole ExactAUC call, at configs[3] (2^24 @ 1 %) and configs[4] (2^27 @ 0.1 %)."""
    from distributedauc_amd.auc import ExactAUC
    from distributedauc_amd.loader import synthetic_scores

    for log2n, pr in ((24, 0.01), (27, 0.001)):
        n = 1 << log2n
        s, y = synthetic_scores(n, pr, dev)
        ms = timeit_b2b(lambda: ops.compact_positives(s, y), reps)
        emit(kernel="compact_positives", log2n=log2n, us=ms * 1e3, label_GBps=n / ms / 1e6)
        ms = timeit_b2b(lambda: ops.split_scores(s, y, negatives=False), reps)
        emit(kernel="split_scores_posonly", log2n=log2n, us=ms * 1e3)
        pos, st = ops.compact_positives(s, y)
        P = int(st[0].item())
        wt = torch.zeros(3, dtype=torch.int64, device=dev)
        ms = timeit_b2b(lambda: ops.auc_counts_sorted_labeled(pos[:P], s, y, 0, n, wt, nonfinite=wt[2:]), reps)
        emit(kernel="sort_plus_query", log2n=log2n, P=P, us=ms * 1e3)
        ev = ExactAUC(method="sort")
        c = ev.counts(y, s)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ev.counts(y, s)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        emit(kernel="exact_auc_sort_eval", log2n=log2n, ms=float(np.median(ts)), ms_min=float(np.min(ts)),
             wins=c["wins"], ties=c["ties"], P=c["P"], N=c["N"])


def bench_paircount(dev, reps, log2n):
    n = 1 << log2n
    g = torch.Generator(device=dev).manual_seed(2024)
    s = torch.rand(n, device=dev, generator=g)
    prate = float(os.environ.get("DAUC_MICRO_POS_RATE", "0.01"))
    y = torch.where(torch.rand(n, device=dev, generator=g) < prate, 1, -1).to(torch.int8)
    pos, neg, st = ops.split_scores(s, y)
    P, N = st[0].item(), st[1].item()
    pos, neg = pos[:P].contiguous(), neg[:N].contiguous()
    med, _ = timeit(lambda: ops.split_scores(s, y), reps)
    emit(kernel="split_scores", n=n, us=med * 1e3, GBps=(n * 5 * 2 + n * 4) / med / 1e6)
    wt = torch.zeros(2, dtype=torch.int64, device=dev)
    ops.auc_counts_sorted(pos, neg, wt)
    sorted_counts = tuple(wt.tolist())
    med, mn = timeit(lambda: ops.auc_counts_sorted(pos, neg, wt), reps * 5)
    emit(kernel="auc_counts_sorted", P=P, N=N, us=med * 1e3, us_min=mn * 1e3,
         effective_pairs_per_s=P * N / med * 1e3, keys_GBps=N * 4 * 12 / med / 1e6)
    if os.environ.get("DAUC_MICRO_SORT_ONLY"):
        return
    ref = sorted_counts
    for v in range(12):
        wt = torch.zeros(2, dtype=torch.int64, device=dev)
        ops.pair_count(pos, neg, wt, variant=v)
        c = tuple(wt.tolist())
        ref = ref or c
        med, mn = timeit(lambda: ops.pair_count(pos, neg, wt, variant=v), reps, warm=1)
        emit(kernel="pair_count", variant=v, P=P, N=N, ms=med, pairs_per_s=P * N / med * 1e3,
             frac_valu=P * N / med * 1e3 / 2.62e13, counts_equal=c == ref)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="update,copy,surrogate,paircount")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--log2n", type=int, default=24)
    ap.add_argument("--variants", default=None, help="comma list of update variants (default: all)")
    ap.add_argument("--sur-variants", default="0", help="comma list of surrogate variants")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = a.which.split(",")
    if "update" in w:
        bench_update(dev, a.reps, [int(v) for v in a.variants.split(",")] if a.variants else range(8))
    if "copy" in w:
        bench_copy(dev, a.reps)
    if "surrogate" in w:
        bench_surrogate(dev, a.reps, [int(v) for v in a.sur_variants.split(",")])
    if "surrogate_b2b" in w:
        bench_surrogate_b2b(dev, a.reps, [int(v) for v in a.sur_variants.split(",")])
    if "aucsort" in w:
        bench_aucsort(dev, a.reps)
    if "paircount" in w:
        bench_paircount(dev, max(3, a.reps // 10), a.log2n)
