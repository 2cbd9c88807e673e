"""What tie-heavy scores cost the one-call exact AUC: per score distribution, the verdict the
enqueued evaluation reports (1: the count index held the table; 2: it refused it, and the blocking
call re-runs the sorted path) and the wall time of the blocking call (dauc_auc_eval_counts, host
read included, mean of `reps` after a warm call). Distributions at 2^24 @ 1 % and 2^27 @ 0.1 %:
U(0,1) (the bench's), U(0,1) rounded to bf16, to 1e-3, 1e-4 and 1e-5, and sigmoid of N(0, 2) logits
rounded to bf16 (a bf16 model's probabilities).

    python scripts/probe_eval_ties.py [reps] [--only DIST LOG2N]   (--only: one case, for a kernel trace)
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else 10
only = None
if "--only" in sys.argv:
    i = sys.argv.index("--only")
    only = (sys.argv[i + 1], int(sys.argv[i + 2]))
dev = torch.device("cuda", 0)


def dists(s):
    g = torch.Generator(device=dev).manual_seed(7)
    yield "uniform", s
    yield "bf16", s.bfloat16().float()
    yield "round1e-3", torch.round(s * 1e3) / 1e3
    yield "round1e-4", torch.round(s * 1e4) / 1e4
    yield "round1e-5", torch.round(s * 1e5) / 1e5
    z = torch.randn(s.numel(), generator=g, device=dev) * 2.0
    yield "sigmoid_bf16_logits", torch.sigmoid(z.bfloat16().float())


for log2n, pr in ((24, 0.01), (27, 0.001)):
    if only and only[1] != log2n:
        continue
    s0, y = synthetic_scores(1 << log2n, pr, dev)
    rec = torch.zeros(8, dtype=torch.int64, device=dev)
    for name, s in dists(s0):
        if only and only[0] != name:
            continue
        s = s.contiguous()
        ops.auc_eval_enqueue(s, y, 0, 1, out=rec)
        verdict = int(rec[7].item())
        c = ops.auc_eval_counts(s, y)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            c = ops.auc_eval_counts(s, y)
        ms = (time.perf_counter() - t0) * 1e3 / reps
        print(json.dumps({"log2n": log2n, "dist": name, "distinct_pos": int(torch.unique(s[y == 1]).numel()),
                          "P": c[2], "verdict": verdict, "ms_blocking_call": ms}), flush=True)
        del s
    del s0, y
    torch.cuda.empty_cache()
