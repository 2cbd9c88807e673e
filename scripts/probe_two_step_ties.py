"""Per-rank device time of the two-step evaluation on tie-heavy scores (bf16-rounded configs[3] /
configs[4]) at G = 8, one GPU: step 1 + step 2 (which reports verdict 2), then the verdict-2 path --
dauc_auc_eval_query_part_sorted over the gathered slots (round 6) vs the whole-vector blocking
dauc_auc_eval_counts_part (before). HIP events around `reps` back-to-back sequences (the blocking
call's host readbacks included in its figure); the parts' counts checked against the one-call
evaluation's.

    python scripts/probe_two_step_ties.py [reps]
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)


def dev_ms(fn):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


G = 8
for log2n, pr in ((24, 0.01), (27, 0.001)):
    s, y = synthetic_scores(1 << log2n, pr, dev)
    s = s.bfloat16().float().contiguous()
    n = s.numel()
    whole = ops.auc_eval_counts(s, y)
    P = whole[2]
    nb = ops.auc_slot_bytes(n, G)
    slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
    mine = torch.empty(nb, dtype=torch.uint8, device=dev)
    rec = torch.zeros(8, dtype=torch.int64, device=dev)
    for r in range(G):
        ops.auc_eval_compact_part(s, y, r, G, slots[r * nb:(r + 1) * nb])
    W = T = 0
    for r in range(G):
        v = ops.auc_eval_query_part_sorted(s, y, r, G, slots, P, out=rec).tolist()
        assert v[7] == 1, v
        W, T = W + v[0], T + v[1]
    pc = torch.zeros(3, dtype=torch.int64, device=dev)

    def steps():
        ops.auc_eval_compact_part(s, y, 0, G, mine)
        ops.auc_eval_query_part(s, y, 0, G, slots, out=rec)

    t12 = dev_ms(steps)
    t_sorted = dev_ms(lambda: ops.auc_eval_query_part_sorted(s, y, 0, G, slots, P, out=rec))
    t_whole = dev_ms(lambda: ops.auc_eval_counts_part(s, y, 0, G, pc))
    print(json.dumps({"log2n": log2n, "G": G, "P": P, "sum_matches_whole": (W, T) == whole[:2],
                      "ms_step1_step2": t12, "ms_query_part_sorted": t_sorted, "ms_counts_part_blocking": t_whole,
                      "per_rank_new": t12 + t_sorted, "per_rank_before": t12 + t_whole}), flush=True)
    del s, y
    torch.cuda.empty_cache()
