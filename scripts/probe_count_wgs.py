"""The two-step's slotted count pass with another number of workgroups (tuning build, DAUC_SLOT_COUNT_WGS
read per launch; each workgroup recomputes the plan from the gathered slots' histograms: fewer read
less, more hold fewer keys each): rank 0's step 1 + step 2 at G = 8 (HIP events around `reps` back-to-back pairs, step 1
alone subtracted), 2^24 @ 1 % and 2^27 @ 0.1 %, the knob interleaved (0 = the product's grid, one
workgroup per 1,024 keys of capacity); the parts' counts checked against the one-call evaluation.

    python scripts/probe_count_wgs.py [reps]
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
dev = torch.device("cuda", 0)


def dev_ms(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with _lib.using(_lib.tuning()):
    G = 8
    for log2n, pr in ((24, 0.01), (27, 0.001)):
        s, y = synthetic_scores(1 << log2n, pr, dev)
        n = s.numel()
        whole = ops.auc_eval_counts(s, y)
        nb = ops.auc_slot_bytes(n, G)
        slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
        mine = torch.empty(nb, dtype=torch.uint8, device=dev)
        rec = torch.zeros(8, dtype=torch.int64, device=dev)
        for r in range(G):
            ops.auc_eval_compact_part(s, y, r, G, slots[r * nb:(r + 1) * nb])
        for rep in range(3):
            for wgs in ("0", "256", "512", "1024", "64"):
                os.environ["DAUC_SLOT_COUNT_WGS"] = wgs
                W = T = 0
                for r in range(G):
                    ops.auc_eval_compact_part(s, y, r, G, mine)
                    v = ops.auc_eval_query_part(s, y, r, G, slots, out=rec).tolist()
                    W, T = W + v[0], T + v[1]
                pair = dev_ms(lambda: (ops.auc_eval_compact_part(s, y, 0, G, mine),
                                       ops.auc_eval_query_part(s, y, 0, G, slots, out=rec)))
                comp = dev_ms(lambda: ops.auc_eval_compact_part(s, y, 0, G, mine))
                print(json.dumps({"log2n": log2n, "wgs": int(wgs), "rep": rep, "match": (W, T) == whole[:2],
                                  "ms_part0": pair, "ms_step2": pair - comp}), flush=True)
        os.environ.pop("DAUC_SLOT_COUNT_WGS", None)
        del s, y
        torch.cuda.empty_cache()
