"""A/B of the one-call evaluation's query paths (tuning build, dauc_set_query_path): 1 = the count
index with per-query window gathers, 2 = the range-slot index. configs[3] (2^24 @ 1 %) and
configs[4] (2^27 @ 0.1 %): wall time of the blocking call (median of `reps`, paths interleaved
per round) and the integers of both paths compared. One JSON line per (n, path).
    python scripts/ab_eval_paths.py [reps] [rounds] [log2n:p,...]
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributedauc_amd import _lib, ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cases = [(int(a), float(b)) for a, b in (c.split(":") for c in (sys.argv[3] if len(sys.argv) > 3 else
                                                                  "27:0.001,24:0.01").split(","))]
dev = torch.device("cuda", 0)
with _lib.using(_lib.tuning()):
    for log2n, pr in cases:
        s, y = synthetic_scores(1 << log2n, pr, dev)
        res = {}
        ts = {1: [], 2: []}
        for _ in range(rounds):
            for path in (1, 2):
                ops.set_query_path(path)
                res[path] = ops.auc_eval_counts(s, y)
                torch.cuda.synchronize()
                for _ in range(reps):
                    t0 = time.perf_counter()
                    ops.auc_eval_counts(s, y)
                    ts[path].append(time.perf_counter() - t0)
        ops.set_query_path(1)
        for path in (1, 2):
            print(json.dumps({"log2n": log2n, "pos": pr, "path": path, "ms_median": float(np.median(ts[path])) * 1e3,
                              "ms_min": float(np.min(ts[path])) * 1e3, "counts": list(res[path]),
                              "equal": res[1] == res[2]}), flush=True)
