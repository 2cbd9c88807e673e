"""Per-rank device time of the two-step sharded evaluation, on ONE GPU.

One rank of a G-GPU job runs dauc_auc_eval_compact_part over its slice, the slot all-gather, and
dauc_auc_eval_query_part over the next slice. Here the G slots are gathered by a device copy once,
and the rank's two calls are timed back to back (HIP events on the stream around `reps` sequences,
no host read in between: the GPU time a rank spends; the collectives are not on one GPU). Step 2
consumes the build state its step 1 prepares in the workspace, so every timed step 2 follows its
step 1 (the step-2 figure is the pair minus step 1 alone). Parts 0 and G-1 at configs[3] (2^24 @
1 %) and configs[4] (2^27 @ 0.1 %), G = 2, 4, 8; the parts' counts are checked against the one-call
evaluation. --ab: the tuning build, step 2's two forms interleaved (dauc_set_index_form: 0 the
slotted build = the product's, 1 round 5's direct build). --base=PATH: the product library and a
baseline build of it (e.g. the previous commit's sources) interleaved, G = 8 only ("lib" in the
line). One JSON line per (n, G, form). With --trace only the G = 8 sequences run (for a rocprofv3
kernel trace of one rank's chain).

    python scripts/probe_two_step.py [reps] [--trace] [--ab | --tuning | --base=PATH]
"""
from __future__ import annotations

import contextlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import _lib, ops  # noqa: E402
from distributedauc_amd.loader import synthetic_scores  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
reps = int(args[0]) if args else 50
trace = "--trace" in sys.argv
ab = "--ab" in sys.argv
tun = ab or "--tuning" in sys.argv  # --tuning: the tuning build, product form (its DAUC_* env knobs)
base = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--base=")), None)
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


ctx = _lib.using(_lib.tuning()) if tun else contextlib.nullcontext()
libs = {"product": None}
if base:
    import ctypes
    libs = {"base": _lib._attach(ctypes.CDLL(base)), "product": None}
with ctx:
    for log2n, pr in ((24, 0.01), (27, 0.001)):
        s, y = synthetic_scores(1 << log2n, pr, dev)
        n = s.numel()
        whole = ops.auc_eval_counts(s, y)
        for G, form, lib in [(G, f, L) for G in ((8,) if trace or base else (2, 4, 8))
                             for f in ((1, 0, 1, 0) if ab else (0,) if tun else (None,))
                             for L in (["base", "product", "base", "product"] if base else ["product"])]:
            if base:  # the libraries' workspace layouts differ: fresh zero-filled workspaces per switch
                ops.workspaces._ws.clear()
            lctx = _lib.using(libs[lib]) if libs[lib] is not None else contextlib.nullcontext()
            with lctx:
                if form is not None:
                    ops.set_index_form(form)
                nb = ops.auc_slot_bytes(n, G)
                slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
                mine = torch.empty(nb, dtype=torch.uint8, device=dev)
                rec = torch.zeros(8, dtype=torch.int64, device=dev)
                for r in range(G):
                    ops.auc_eval_compact_part(s, y, r, G, slots[r * nb:(r + 1) * nb])
                W = T = 0
                for r in range(G):
                    ops.auc_eval_compact_part(s, y, r, G, mine)
                    v = ops.auc_eval_query_part(s, y, r, G, slots, out=rec).tolist()
                    assert v[4] == 0 and v[7] == 1, v
                    W, T = W + v[0], T + v[1]
                out = {"log2n": log2n, "G": G, "form": form, "lib": lib, "slot_bytes": nb, "sum_matches_whole": (W, T) == whole[:2]}
                for r in (0, G - 1):
                    out[f"ms_part{r}"] = dev_ms(lambda: (ops.auc_eval_compact_part(s, y, r, G, mine),
                                                         ops.auc_eval_query_part(s, y, r, G, slots, out=rec)))
                    out[f"ms_compact_part{r}"] = dev_ms(lambda: ops.auc_eval_compact_part(s, y, r, G, mine))
                    out[f"ms_query_part{r}"] = out[f"ms_part{r}"] - out[f"ms_compact_part{r}"]
                out["env"] = {k: v for k, v in os.environ.items() if k.startswith("DAUC_")}
                if G == 8:  # the one-call evaluation (enqueue, part 0 of 1) on the same data, this form
                    out["ms_whole_one_call_events"] = dev_ms(lambda: ops.auc_eval_enqueue(s, y, 0, 1, out=rec))
                    assert tuple(rec.tolist()[:2]) == whole[:2] and rec.tolist()[7] == 1
                print(json.dumps(out), flush=True)
        del s, y
        torch.cuda.empty_cache()
    if tun:
        ops.set_index_form(0)
