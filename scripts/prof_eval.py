"""A short exact-AUC run for profilers: `reps` one-call evaluations of 2^log2n synthetic scores
(the bench's generator) after one warm call.
    python scripts/prof_eval.py [log2n] [pos] [reps]
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd.auc import ExactAUC  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 27
pos = float(sys.argv[2]) if len(sys.argv) > 2 else 0.001
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda", 0)
s, y = synthetic_scores(1 << log2n, pos, dev)
ev = ExactAUC(method="sort")
c = ev.counts(y, s)
for _ in range(reps):
    c = ev.counts(y, s)
torch.cuda.synchronize()
print(c, flush=True)
