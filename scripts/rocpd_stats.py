"""Per-kernel duration summary of a rocprofv3 --kernel-trace database (rocpd sqlite output).

Groups dispatches by (short kernel name, grid size) and prints count, mean / min / max / total
microseconds, sorted by total time. Optional substring filter on the name.

    python scripts/rocpd_stats.py gpurun_out/x/prof/run_results.db [name-filter] [--json out.json]
"""
from __future__ import annotations

import json
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)                     # drop the parameter list
    n = re.sub(r"<.*>", "<>", n)                   # template args
    return n[-90:]


def summary(db: str, filt: str = ""):
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, grid_y, workgroup_x, duration from kernels").fetchall()
    g = defaultdict(list)
    for name, gx, gy, wx, dur in rows:
        if filt and filt not in name:
            continue
        g[(short(name), gx // max(wx, 1), gy)].append(dur / 1e3)
    out = []
    for (name, blocks, gy), d in g.items():
        out.append({"kernel": name, "workgroups": blocks * gy, "calls": len(d), "mean_us": sum(d) / len(d),
                    "min_us": min(d), "max_us": max(d), "total_us": sum(d)})
    return sorted(out, key=lambda r: -r["total_us"])


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    res = summary(args[0], args[1] if len(args) > 1 else "")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(res, f, indent=1)
    for r in res[:40]:
        print(f"{r['total_us']:10.1f} {r['calls']:5d} {r['mean_us']:9.2f} {r['min_us']:9.2f} {r['max_us']:9.2f} "
              f"{r['workgroups']:7d}  {r['kernel']}")
