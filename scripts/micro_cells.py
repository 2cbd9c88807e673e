"""Search-structure A/B for the sort method: the labeled query pass and the one-call evaluation
at configs[3] (2^24 @ 1 %) and configs[4] (2^27 @ 0.1 %) in each dauc_set_search_mode
(0 automatic, 1 tree), HIP events on the launch stream, same counts required. Every call runs in
the tuning build, whose search mode the switch sets (the product library ignores it).
One JSON line per (config, mode)."""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import _lib, ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
modes = [int(m) for m in (sys.argv[2] if len(sys.argv) > 2 else "1,0").split(",")]
dev = torch.device("cuda", 0)
_tuning = _lib.using(_lib.tuning())
_tuning.__enter__()
for log2n, pr in ((24, 0.01), (27, 0.001)):
    n = 1 << log2n
    s, y = synthetic_scores(n, pr, dev)
    pos, st = ops.compact_positives(s, y)
    P = int(st[0].item())
    ref = None
    for m in modes:
        ops.set_search_mode(m)
        wt = torch.zeros(3, dtype=torch.int64, device=dev)
        for _ in range(3):
            wt.zero_()
            ops.auc_counts_sorted_labeled(pos[:P], s, y, 0, n, wt, nonfinite=wt[2:])
        counts = wt.tolist()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ops.auc_counts_sorted_labeled(pos[:P], s, y, 0, n, wt, nonfinite=wt[2:])
        e1.record()
        e1.synchronize()
        q_us = e0.elapsed_time(e1) / reps * 1e3
        for _ in range(3):
            c = ops.auc_eval_counts(s, y)
        e0.record()
        for _ in range(reps):
            c = ops.auc_eval_counts(s, y)
        e1.record()
        e1.synchronize()
        ev_us = e0.elapsed_time(e1) / reps * 1e3
        ref = ref or counts
        rec = {"log2n": log2n, "pos": pr, "P": P, "mode": m, "sorted_labeled_us": q_us, "eval_us": ev_us,
               "counts": counts, "eval_counts": list(c[:2]), "agree": counts == ref and list(c[:2]) == counts[:2]}
        print(json.dumps(rec), flush=True)
ops.set_search_mode(0)
_tuning.__exit__(None, None, None)
