"""A/B of the exact-AUC evaluation across library builds (DAUC_LIB selects the build).

One JSON line per (size, measurement): the one-call evaluation's median wall time at configs[3]
(2^24 @ 1 %) and configs[4] (2^27 @ 0.1 %), with its integer counts (they must agree across
builds), plus the first call (cold: workspace allocation included) and calls alternating between
two different test sets of the same length.
    DAUC_LIB=tuning/libdauc_x.so python scripts/ab_eval.py [reps] [tag]
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributedauc_amd.auc import ExactAUC  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
tag = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(os.environ.get("DAUC_LIB", "libdauc.so"))
dev = torch.device("cuda", 0)


def wall(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, r


for log2n, pr in ((24, 0.01), (27, 0.001)):
    n = 1 << log2n
    s, y = synthetic_scores(n, pr, dev)
    ev = ExactAUC(method="sort")
    cold, c = wall(lambda: ev.counts(y, s))
    ts = [wall(lambda: ev.counts(y, s))[0] for _ in range(reps)]
    # a second test set of the same length (other seed, other P): alternate the two
    g = torch.Generator(device=dev).manual_seed(99)
    s2 = torch.rand(n, device=dev, generator=g)
    y2 = torch.where(torch.rand(n, device=dev, generator=g) < pr * 1.1, 1, -1).to(torch.int8)
    alt = []
    for k in range(reps):
        alt.append(wall(lambda: ev.counts(y2 if k % 2 == 0 else y, s2 if k % 2 == 0 else s))[0])
    print(json.dumps({"lib": tag, "log2n": log2n, "ms": float(np.median(ts)) * 1e3, "ms_min": float(np.min(ts)) * 1e3,
                      "ms_cold": cold * 1e3, "ms_alternating": float(np.median(alt)) * 1e3,
                      "wins": c["wins"], "ties": c["ties"], "P": c["P"], "N": c["N"]}), flush=True)
