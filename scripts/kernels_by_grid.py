"""Per (kernel, grid size) launch statistics of this library's kernels from a rocprofv3 kernel trace
(the `dauc_kernels_by_grid.json` of profiles/rNN/final): calls, mean / median / min duration in us.

    python scripts/kernels_by_grid.py <trace dir or kernel_trace.csv> <out.json>
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import statistics
import sys

PREFIXES = ("void dauc::(anonymous namespace)::", "dauc::(anonymous namespace)::")


def short(name: str) -> str | None:
    for p in PREFIXES:
        if name.startswith(p):
            return name[len(p):].split("(")[0]
    return None


def main(src: str, dst: str) -> None:
    files = [src] if src.endswith(".csv") else glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
    per = collections.defaultdict(list)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if k is None:
                    continue
                grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
                per[(k, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    out = [{"kernel": k, "grid_threads": g, "calls": len(v), "mean_us": statistics.fmean(v),
            "median_us": statistics.median(v), "min_us": min(v)} for (k, g), v in sorted(per.items())]
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"{len(out)} entries -> {dst}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
