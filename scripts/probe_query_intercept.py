"""The query pass's fixed cost: rank 0's dauc_auc_eval_query_part at configs[4] (2^27 @ 0.1 %) for
G = 8 .. 1024 parts (2^24 .. 2^17 queries over the same table), `reps` times each; run under
`rocprofv3 --kernel-trace` and read query_ci_kernel's duration per G (the gather's grid.y is G).
    python scripts/probe_query_intercept.py [reps] [positive fraction]
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
pos = float(sys.argv[2]) if len(sys.argv) > 2 else 0.001  # a smaller table: a smaller LDS index
dev = torch.device("cuda", 0)
s, y = synthetic_scores(1 << 27, pos, dev)
n = s.numel()
rec = torch.zeros(8, dtype=torch.int64, device=dev)
for G in (8, 16, 32, 64, 128, 256, 1024):
    nb = ops.auc_slot_bytes(n, G)
    slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
    for r in range(G):
        ops.auc_eval_compact_part(s, y, r, G, slots[r * nb:(r + 1) * nb])
    for _ in range(reps):
        ops.auc_eval_query_part(s, y, 0, G, slots, out=rec)
    torch.cuda.synchronize()
    print(G, rec.tolist(), flush=True)
