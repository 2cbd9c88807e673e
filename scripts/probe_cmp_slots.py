"""The unordered compaction's tile size (tuning build, DAUC_CMP_SLOTS: label groups of 16 per thread
of a 256-thread workgroup, 8 / 16 / 32 / 64; the product takes 32 from 2^25 labels, else 8): one rank's
step 1 at G = 8 (dauc_auc_eval_compact_part over a 2^21 / 2^24-label slice) and the one-call
evaluation (enqueue) at 2^24 @ 1 % and 2^27 @ 0.1 %, HIP events around `reps` back-to-back calls,
the sizes interleaved three times; the one-call counts checked against the product's.

    python scripts/probe_cmp_slots.py [reps]
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
        mine = torch.empty(nb, dtype=torch.uint8, device=dev)
        rec = torch.zeros(8, dtype=torch.int64, device=dev)
        for rep in range(3):
            for sl in ("0", "8", "16", "32", "64"):
                os.environ["DAUC_CMP_SLOTS"] = sl
                ops.auc_eval_enqueue(s, y, 0, 1, out=rec)
                ok = tuple(rec.tolist()[:2]) == whole[:2]
                print(json.dumps({"log2n": log2n, "slots": int(sl), "rep": rep, "counts_ok": ok,
                                  "ms_compact_part0": dev_ms(lambda: ops.auc_eval_compact_part(s, y, 0, G, mine)),
                                  "ms_one_call": dev_ms(lambda: ops.auc_eval_enqueue(s, y, 0, 1, out=rec))}),
                      flush=True)
        os.environ.pop("DAUC_CMP_SLOTS", None)
        del s, y
        torch.cuda.empty_cache()
