"""The distinct-key query pass alone (tuning build, search mode 2: the sorted path builds the
distinct-key index, the tree and count-index passes return at once), HIP events around `reps`
back-to-back dauc_auc_counts_sorted_labeled calls on bf16-rounded scores at 2^24 @ 1 % and
2^27 @ 0.1 %. (It interleaved DAUC_DK_U = 2 and 4 float4 slots per iteration while that knob existed:
4 spills and was removed; the second leg of each pair now runs the product's 2 again.) Counts
checked equal.

    python scripts/probe_dk_query.py [reps]
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import _lib, ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)

with _lib.using(_lib.tuning()):
    ops.set_search_mode(2)
    for log2n, pr in ((24, 0.01), (27, 0.001)):
        s0, y = synthetic_scores(1 << log2n, pr, dev)
        s = s0.bfloat16().float().contiguous()
        pos = s[y == 1].contiguous()
        ref = None
        for rep in range(3):
            for u in ("2", "4"):
                os.environ["DAUC_DK_U"] = u
                wt = torch.zeros(3, dtype=torch.int64, device=dev)
                fn = lambda: ops.auc_counts_sorted_labeled(pos, s, y, 0, s.numel(), wt, nonfinite=wt[2:])  # noqa: E731
                wt.zero_()
                fn()
                got = tuple(wt.tolist())
                ref = ref or got
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                print(json.dumps({"log2n": log2n, "U": int(u), "rep": rep, "same": got == ref,
                                  "ms_sorted_path": e0.elapsed_time(e1) / reps}), flush=True)
        os.environ.pop("DAUC_DK_U", None)
    ops.set_search_mode(0)
