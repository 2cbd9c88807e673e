"""A/B of the compaction's staged-score variant (tuning build, dauc_set_compact_stage): device time (HIP events
around `reps` back-to-back enqueued calls) of rank 0's dauc_auc_eval_compact_part and two-step
sequence at G = 8, and of the one-call dauc_auc_eval_enqueue (G = 1), at configs[3] (2^24 @ 1 %)
and configs[4] (2^27 @ 0.1 %), with the staged-score variant off (0) and on (1)
(include/dauc_tuning.h). One JSON line per (n, stage).
    python scripts/ab_compact_stage.py [reps] [0,1]
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import _lib, ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ts = [int(t) for t in (sys.argv[2] if len(sys.argv) > 2 else "0,1,0,1").split(",")]
dev = torch.device("cuda", 0)


def dev_ms(fn):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with _lib.using(_lib.tuning()):
    for log2n, pr in ((24, 0.01), (27, 0.001)):
        s, y = synthetic_scores(1 << log2n, pr, dev)
        n, G = s.numel(), 8
        nb = ops.auc_slot_bytes(n, G)
        rec = torch.zeros(8, dtype=torch.int64, device=dev)
        ref = None
        for t in ts:
            ops.set_compact_stage(t)
            slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
            for r in range(G):
                ops.auc_eval_compact_part(s, y, r, G, slots[r * nb:(r + 1) * nb])
            recs = [ops.auc_eval_query_part(s, y, r, G, slots).tolist() for r in range(G)]
            one = ops.auc_eval_enqueue(s, y, 0, 1).tolist()
            got = (sum(v[0] for v in recs), sum(v[1] for v in recs), one[0], one[1])
            ref = ref or got
            mine = slots[:nb]
            d_cp = dev_ms(lambda: ops.auc_eval_compact_part(s, y, 0, G, mine))
            d_two = dev_ms(lambda: (ops.auc_eval_compact_part(s, y, 0, G, mine),
                                    ops.auc_eval_query_part(s, y, 0, G, slots, out=rec)))
            d_one = dev_ms(lambda: ops.auc_eval_enqueue(s, y, 0, 1, out=rec))
            print(json.dumps({"log2n": log2n, "stage": t, "ms_compact_part_g8": d_cp, "ms_two_step_g8": d_two,
                              "ms_enqueue_g1": d_one, "counts": got, "equal": got == ref}), flush=True)
        ops.set_compact_stage(0)
