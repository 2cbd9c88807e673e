"""Timing ablations of the two-step's slotted step 2 (tuning build; DAUC_QUERY_ABL selects one;
the counts are wrong by design for ABL != 0, so they are not checked): rank 0's step 1 + step 2 at
G = 8, 2^24 @ 1 % and 2^27 @ 0.1 %, HIP events around back-to-back pairs, step 1 alone subtracted.
One JSON line per size. python scripts/probe_query_abl.py [reps]"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import _lib, ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
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
    ops.set_index_form(0)
    G = 8
    for log2n, pr in ((24, 0.01), (27, 0.001)):
        s, y = synthetic_scores(1 << log2n, pr, dev)
        n = s.numel()
        nb = ops.auc_slot_bytes(n, G)
        slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
        mine = torch.empty(nb, dtype=torch.uint8, device=dev)
        rec = torch.zeros(8, dtype=torch.int64, device=dev)
        for r in range(G):
            ops.auc_eval_compact_part(s, y, r, G, slots[r * nb:(r + 1) * nb])
        pair = dev_ms(lambda: (ops.auc_eval_compact_part(s, y, 0, G, mine),
                               ops.auc_eval_query_part(s, y, 0, G, slots, out=rec)))
        comp = dev_ms(lambda: ops.auc_eval_compact_part(s, y, 0, G, mine))
        print(json.dumps({"log2n": log2n, "abl": os.environ.get("DAUC_QUERY_ABL", "0"), "ms_pair": pair,
                          "ms_compact": comp, "ms_step2": pair - comp}), flush=True)
        del s, y
        torch.cuda.empty_cache()
