"""The one-call exact-AUC evaluation at configs[4] (2^27 scores, 0.1 % positives), `calls` times:
the program rocprofv3 --pmc passes profile (scripts/gpu_r03f.sh)."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd.auc import ExactAUC  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 5
log2n = int(sys.argv[2]) if len(sys.argv) > 2 else 27
dev = torch.device("cuda", 0)
s, y = synthetic_scores(1 << log2n, 0.001 if log2n == 27 else 0.01, dev)
ev = ExactAUC(method="sort")
for _ in range(calls):
    c = ev.counts(y, s)
torch.cuda.synchronize()
print(c)
