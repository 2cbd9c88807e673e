"""Per-rank cost of the sharded sort-method evaluation on ONE GPU: dauc_auc_eval_counts_part for
part 0 and part G-1 of G (what one rank of a G-GPU job runs before its all-reduce), next to the
whole-vector dauc_auc_eval_counts, at configs[3] (2^24 @ 1 %) and configs[4] (2^27 @ 0.1 %).
Wall time of the blocking call (median of `reps`), and the parts' counts summed against the
whole call's. One JSON line per (n, G)."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributedauc_amd import ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda", 0)
pc = torch.zeros(3, dtype=torch.int64, device=dev)


def wall(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


for log2n, pr in ((24, 0.01), (27, 0.001)):
    s, y = synthetic_scores(1 << log2n, pr, dev)
    whole = ops.auc_eval_counts(s, y)
    t_whole = wall(lambda: ops.auc_eval_counts(s, y))
    print(json.dumps({"log2n": log2n, "G": 1, "fn": "dauc_auc_eval_counts", "ms": t_whole, "W": whole[0],
                      "T": whole[1]}), flush=True)
    for G in (2, 4, 8):
        W = T = 0
        for r in range(G):
            o = ops.auc_eval_counts_part(s, y, r, G, pc)
            W, T = W + o[0], T + o[1]
        t0 = wall(lambda: ops.auc_eval_counts_part(s, y, 0, G, pc))
        tl = wall(lambda: ops.auc_eval_counts_part(s, y, G - 1, G, pc))
        print(json.dumps({"log2n": log2n, "G": G, "fn": "dauc_auc_eval_counts_part", "ms_part0": t0,
                          "ms_last": tl, "sum_matches_whole": (W, T) == (whole[0], whole[1])}), flush=True)
        # the sharded path's own call: the part enqueued with no host sync, then the one read of its
        # 64-byte record (ExactAUC reads the all-gathered records instead)
        rec = torch.zeros(8, dtype=torch.int64, device=dev)
        W = T = 0
        for r in range(G):
            v = ops.auc_eval_enqueue(s, y, r, G, out=rec).tolist()
            W, T = W + v[0], T + v[1]
        e0 = wall(lambda: ops.auc_eval_enqueue(s, y, 0, G, out=rec).tolist())
        el = wall(lambda: ops.auc_eval_enqueue(s, y, G - 1, G, out=rec).tolist())
        print(json.dumps({"log2n": log2n, "G": G, "fn": "dauc_auc_eval_enqueue + record read", "ms_part0": e0,
                          "ms_last": el, "sum_matches_whole": (W, T) == (whole[0], whole[1])}), flush=True)
        # round 4: the two-step form -- the rank compacts its slice into its slot, the slots are
        # all-gathered (a device copy here, one GPU), it counts its query range from the gathered
        # table; per rank: its own compaction + its query part + the record read (the two
        # collectives are not on one GPU)
        n = s.numel()
        nb = ops.auc_slot_bytes(n, G)
        slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
        mine = torch.empty(nb, dtype=torch.uint8, device=dev)
        for r in range(G):
            ops.auc_eval_compact_part(s, y, r, G, mine)
            slots[r * nb:(r + 1) * nb].copy_(mine)
        W = T = 0
        for r in range(G):
            v = ops.auc_eval_query_part(s, y, r, G, slots, out=rec).tolist()
            W, T = W + v[0], T + v[1]

        def two_step(r):
            ops.auc_eval_compact_part(s, y, r, G, mine)
            return ops.auc_eval_query_part(s, y, r, G, slots, out=rec).tolist()

        t0 = wall(lambda: two_step(0))
        tl = wall(lambda: two_step(G - 1))
        print(json.dumps({"log2n": log2n, "G": G, "fn": "two-step: compact_part + query_part + record read",
                          "ms_part0": t0, "ms_last": tl, "slot_bytes": nb,
                          "sum_matches_whole": (W, T) == (whole[0], whole[1])}), flush=True)

        # device time per rank (HIP events on the stream around `reps` back-to-back enqueued
        # sequences, no host read in between): what a rank's GPU spends; the wall times above also
        # hold the Python binding's calls and the record read
        def dev_ms(fn):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps

        d_enq = dev_ms(lambda: ops.auc_eval_enqueue(s, y, 0, G, out=rec))
        d_two = dev_ms(lambda: (ops.auc_eval_compact_part(s, y, 0, G, mine),
                                ops.auc_eval_query_part(s, y, 0, G, slots, out=rec)))
        print(json.dumps({"log2n": log2n, "G": G, "fn": "device time per rank (events)",
                          "ms_enqueue_form": d_enq, "ms_two_step": d_two}), flush=True)
