"""Per-training-step GPU time by kernel family from a rocprofv3 kernel trace of bench.py.

The window is the last N steps before the final update launch (one dauc_pd_update per step) of
the largest model in the trace (the update launches with the largest grid: the default bench also
trains ResNet-18 for its N = 2 leg).

    python scripts/step_breakdown.py gpurun_out/prof_r01/bench_kernel_trace.csv [N]
"""
from __future__ import annotations

import collections
import csv
import sys


def family(name: str) -> str:
    if name.startswith("igemm_fwd"):
        return "miopen fwd"
    if name.startswith("igemm_bwd"):
        return "miopen bwd"
    if name.startswith("igemm_wrw"):
        return "miopen wrw"
    if "Cijk" in name:
        return "hipblaslt"
    if "bn_partial" in name:
        return "bn partial"
    if "bn_elementwise" in name:
        return "bn elementwise"
    return name[:100]


def main(path: str, nsteps: int = 5) -> None:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    grid = lambda r: int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)  # noqa: E731
    upd = [(i, grid(r)) for i, r in enumerate(rows) if "pd_update_kernel" in r["Kernel_Name"]]
    gmax = max(gs for _, gs in upd)
    ups = [i for i, gs in upd if gs == gmax]
    i0, i1 = ups[-1 - nsteps], ups[-1]
    agg: dict = collections.defaultdict(lambda: [0.0, 0])
    busy = 0.0
    for r in rows[i0 + 1:i1 + 1]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / nsteps
        busy += d
        a = agg[family(r["Kernel_Name"])]
        a[0] += d
        a[1] += 1
    span = (int(rows[i1]["End_Timestamp"]) - int(rows[i0]["End_Timestamp"])) / 1e6 / nsteps
    print(f"span {span:.2f} ms/step, kernels busy {busy:.2f} ms/step")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:24]:
        print(f"{t:7.3f} ms {c / nsteps:6.1f}/step  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
