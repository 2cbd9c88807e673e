"""The sort method's kernels at configs[4] (2^27 scores, 0.1 % positives) for rocprofv3:
compaction once, then `reps` sorted-count calls (radix sort of the positives + tree build +
the labeled query kernel). Prints the counts so a profile run is also a parity smoke."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 27
pr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.001
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda", 0)
n = 1 << log2n
s, y = synthetic_scores(n, pr, dev)
pos, st = ops.compact_positives(s, y)
P = int(st[0].item())
for _ in range(reps):
    wt = torch.zeros(3, dtype=torch.int64, device=dev)
    ops.auc_counts_sorted_labeled(pos[:P], s, y, 0, n, wt, nonfinite=wt[2:])
torch.cuda.synchronize()
print("P", P, "counts", wt.tolist())
