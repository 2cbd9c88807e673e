"""HBM bytes per launch of the roofline kernels from rocprofv3 PMC passes -> profiles/traffic.json.

Input: the counter-collection CSVs of scripts/gpu_pmc.sh (one pass per counter, FETCH_SIZE and
WRITE_SIZE, over scripts/micro_kernels.py --which update,surrogate). Corrections, as
MI355X_MICROARCH.md §HBM prescribes for gfx950: both counters are in KB (1024 B); FETCH_SIZE
reports half the bytes of wide (16 B/lane) streaming reads, so it is doubled; WRITE_SIZE is exact
for 16 B/lane stores. Per kernel the median over its dispatches is kept; for the surrogate only the
dispatches with the largest grid (the B = 2^26 launches) are used.

    python scripts/pmc_traffic.py gpurun_out/pmc_r01 profiles/r01
"""
from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys

ALGORITHMIC = {"pd_update": 24 * 23_512_130, "surrogate_2^26": 9 * (1 << 26),
               # configs[4] sort-method passes at 2^27 scores, 0.1 % positives (134,447 of them)
               "compact_count_2^27": (1 << 27) + (1 << 27) // 8,          # labels + 1-bit masks
               "compact_write_2^27": (1 << 27) // 8 + 8 * 134_447,        # masks + positives read & written
               "query_labeled_2^27": 5 * (1 << 27),
               # the count-index query (the default search since round 2): same stream of scores + labels
               "query_ci_2^27": 5 * (1 << 27)}


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def kernel_key(name: str) -> str | None:
    if "pd_update_kernel" in name:
        return "pd_update"
    if "surrogate_rows_reduce_kernel" in name:
        return "surrogate_reduce"
    if ("surrogate_chunk_kernel" in name or "surrogate_kernel" in name or "surrogate_tail_kernel" in name
            or "surrogate_tail_x_kernel" in name):
        return "surrogate"
    if "compact_count_kernel" in name:
        return "compact_count_2^27"
    if "compact_write_kernel" in name:
        return "compact_write_2^27"
    if "query_labeled_kernel" in name:
        return "query_labeled_2^27"
    if "query_ci_kernel" in name:
        return "query_ci_2^27"
    return None


def per_kernel(rs, counter):
    by = {}
    for r in rs:
        if r["Counter_Name"] != counter:
            continue
        k = kernel_key(r["Kernel_Name"])
        if k is None:
            continue
        by.setdefault(k, []).append((int(r["Grid_Size"]), float(r["Counter_Value"]) * 1024.0))
    out = {}
    for k, v in by.items():
        if k.startswith("surrogate"):
            gmax = max(g for g, _ in v)
            v = [x for x in v if x[0] == gmax]
        out[k] = statistics.median(b for _, b in v)
    return out


def main(src: str, dst: str):
    fetch = per_kernel(rows(os.path.join(src, "**", "*FETCH_SIZE*counter_collection.csv")), "FETCH_SIZE")
    write = per_kernel(rows(os.path.join(src, "**", "*WRITE_SIZE*counter_collection.csv")), "WRITE_SIZE")
    res = {
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (scripts/gpu_pmc.sh), "
                  "counter-collection CSV per dispatch; KB = 1024 B; FETCH_SIZE doubled for gfx950 wide streaming "
                  "reads (MI355X_MICROARCH.md §HBM); median over dispatches (surrogate: largest grid = B 2^26, the one-launch tail kernel, or chunk kernel + row-reduce kernel); "
                  "scripts/pmc_traffic.py",
        "source": dst,
    }
    # the surrogate call at large B is two launches: the streaming chunk kernel + the row reduction
    for key in ("surrogate",):
        if key + "_reduce" in fetch and key in fetch:
            fetch[key] += fetch[key + "_reduce"]
        if key + "_reduce" in write and key in write:
            write[key] += write[key + "_reduce"]
    for k, name in (("pd_update", "pd_update"), ("surrogate", "surrogate_2^26")):
        if k in fetch and k in write:
            rd, wr = 2.0 * fetch[k], write[k]
            res[name] = rd + wr
            res[name + "_detail"] = {"read_bytes": rd, "write_bytes": wr}
            res[name + "_algorithmic"] = ALGORITHMIC[name]
    # the exact-AUC passes: the compaction streams labels (16 B per lane) and gathers scores; the query
    # streams float4 + char4 and gathers 16-B buckets from L2 (uncalibrated access widths: the raw
    # FETCH_SIZE is reported next to the doubled one)
    # (with the count index as the search, the tree kernel is enqueued too and returns at once:
    # its entry is kept only when it did the work)
    for k in ("compact_count_2^27", "compact_write_2^27", "query_labeled_2^27", "query_ci_2^27"):
        if k in fetch and k in write and 2.0 * fetch[k] + write[k] > 0.5 * ALGORITHMIC[k]:
            res[k] = 2.0 * fetch[k] + write[k]
            res[k + "_detail"] = {"read_bytes_doubled": 2.0 * fetch[k], "read_bytes_raw": fetch[k],
                                  "write_bytes": write[k]}
            res[k + "_algorithmic"] = ALGORITHMIC[k]
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        stem = os.path.basename(f).replace("_counter_collection.csv", "")
        with open(f) as fh, open(os.path.join(dst, f"{stem}_dauc.csv"), "w", newline="") as oh:
            rd = csv.DictReader(fh)
            w = csv.DictWriter(oh, fieldnames=rd.fieldnames)
            w.writeheader()
            for r in rd:
                if kernel_key(r["Kernel_Name"]):
                    w.writerow(r)
    with open("profiles/traffic.json", "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
