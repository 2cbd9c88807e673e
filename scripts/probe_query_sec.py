"""A/B of the slotted query's secondary-window forms (tuning build, DAUC_QUERY_SEC read per launch):
1 = one secondary window per lane per group (the product's), 0 = one per query (round 6's first
form); DAUC_QUERY_GD=3: form 1 with three groups in flight (windows issued two groups before their
count; measured, then dropped: the knob no longer selects anything). Interleaved (1, GD 2), (0, GD 2),
(1, GD 3), three times, on the same data: the one-call evaluation (enqueue, HIP
events around `reps` back-to-back calls) and rank 0's step 1 + step 2 at G = 8, at configs[3]
(2^24 @ 1 %) and configs[4] (2^27 @ 0.1 %); every form's counts are checked against round 5's
direct build (index form 1). One JSON line per (n, form, rep).

    python scripts/probe_query_sec.py [reps]
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
        ops.set_index_form(1)
        ref = ops.auc_eval_counts(s, y)
        ops.set_index_form(0)
        nb = ops.auc_slot_bytes(n, G)
        slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
        mine = torch.empty(nb, dtype=torch.uint8, device=dev)
        rec = torch.zeros(8, dtype=torch.int64, device=dev)
        for r in range(G):
            ops.auc_eval_compact_part(s, y, r, G, slots[r * nb:(r + 1) * nb])
        for rep in range(3):
            for sec, gd in (("1", "2"), ("0", "2"), ("1", "3")):
                os.environ["DAUC_QUERY_SEC"], os.environ["DAUC_QUERY_GD"] = sec, gd
                whole = ops.auc_eval_counts(s, y)
                W = T = 0
                for r in range(G):
                    ops.auc_eval_compact_part(s, y, r, G, mine)
                    v = ops.auc_eval_query_part(s, y, r, G, slots, out=rec).tolist()
                    assert v[4] == 0 and v[7] == 1, v
                    W, T = W + v[0], T + v[1]
                out = {"log2n": log2n, "sec": int(sec), "GD": int(gd), "rep": rep, "whole_matches": whole[:2] == ref[:2],
                       "parts_match": (W, T) == ref[:2]}
                out["ms_one_call"] = dev_ms(lambda: ops.auc_eval_enqueue(s, y, 0, 1, out=rec))
                pair = dev_ms(lambda: (ops.auc_eval_compact_part(s, y, 0, G, mine),
                                       ops.auc_eval_query_part(s, y, 0, G, slots, out=rec)))
                comp = dev_ms(lambda: ops.auc_eval_compact_part(s, y, 0, G, mine))
                out.update(ms_part0=pair, ms_compact_part0=comp, ms_query_part0=pair - comp)
                print(json.dumps(out), flush=True)
        os.environ.pop("DAUC_QUERY_SEC", None)
        os.environ.pop("DAUC_QUERY_GD", None)
        del s, y
        torch.cuda.empty_cache()
