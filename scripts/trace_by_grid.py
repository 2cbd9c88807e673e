"""Per-(kernel, grid size) durations from a rocprofv3 --kernel-trace CSV.

bench.py runs two model sizes through the same update kernel (ResNet-50 for the headline,
ResNet-18 for configs[0]), so the --stats average mixes them; this splits the libdauc.so
kernels by grid size so the headline launch can be compared with the bench line's HIP-event
figure. Usage: python scripts/trace_by_grid.py <kernel_trace.csv> <out.json>"""
from __future__ import annotations

import collections
import csv
import json
import statistics
import sys


def main(src: str, dst: str) -> None:
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"]
        if "dauc::" not in name:
            continue
        short = name.replace("void ", "").replace("dauc::(anonymous namespace)::", "").split("(")[0]
        d[(short, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = [{"kernel": k, "grid_threads": g, "calls": len(v), "mean_us": statistics.fmean(v),
            "median_us": statistics.median(v), "min_us": min(v)} for (k, g), v in sorted(d.items())]
    json.dump(out, open(dst, "w"), indent=1)
    for o in out:
        print(f"{o['kernel'][:60]:60s} {o['grid_threads']:>10d} {o['calls']:5d} {o['mean_us']:9.2f} {o['median_us']:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
