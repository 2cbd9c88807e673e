"""VALU-issue roofline of the labeled query pass from committed rocprofv3 data.

Inputs (profiles/r02/pmc_count_index/, or the directory given as argv[1], e.g. profiles/r04/pmc_query/
from scripts/gpu_r04_pmcq.sh over the one-call evaluation): SQ_INSTS_VALU /
SQ_INSTS_LDS per dispatch (one --pmc pass, scripts/gpu_pmc_ci.sh) and the kernel's average
duration from a separate --kernel-trace --stats pass over the same command; LDS bank-conflict,
wait and in-flight counters. The query pass is the count-index kernel (query_ci_kernel) where the
table fits it, else the tree kernel (query_labeled_kernel); every dispatch of either is counted.
Peak: 256 CUs x 4 SIMD-32 x 2.4 GHz / 2 cycles per wave64 VALU instruction = 1.2288e12
wave-instructions/s (MI355X_MICROARCH.md, execution model). Writes profiles/query_valu.json,
which bench.py attaches to the AUC records."""
from __future__ import annotations

import collections
import csv
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
SRC = Path(sys.argv[1]) if len(sys.argv) > 1 else REPO / "profiles" / "r02" / "pmc_count_index"
QUERY_KERNELS = ("query_ci_kernel", "query_labeled_kernel")
PEAK = 256 * 4 * 2.4e9 / 2


def counters(f):
    """Per-dispatch counter sums of the query kernel that did the work (the other one of the pair
    returns at once), averaged over its dispatches."""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in QUERY_KERNELS):
            agg[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    by_kernel = collections.defaultdict(list)
    for (name, _), v in agg.items():
        by_kernel[name].append(v)
    vals = max(by_kernel.values(), key=lambda vs: sum(sum(v.values()) for v in vs) / len(vs))
    return {k: sum(v[k] for v in vals) / len(vals) for k in vals[0]}


def avg_us(f):
    best = None
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in QUERY_KERNELS):
            us = float(r["AverageNs"]) / 1e3
            best = us if best is None or us > best else best
    if best is None:
        raise SystemExit(f"no query kernel in {f}")
    return best


def main():
    out = {"method": __doc__.split("\n\n")[1].replace("\n", " "), "peak_wave_instr_per_s": PEAK,
           "source": str(SRC.resolve().relative_to(REPO)) if SRC.resolve().is_relative_to(REPO) else str(SRC)}
    for tag, n in (("27", 1 << 27), ("24", 1 << 24)):
        c = counters(SRC / f"valu{tag}_counters.csv")
        us = avg_us(SRC / f"trace{tag}_kernel_stats.csv")
        rate = c["SQ_INSTS_VALU"] / (us * 1e-6)
        rec = {"queries": n, "avg_launch_us": us, "valu_wave_instr": c["SQ_INSTS_VALU"],
               "valu_per_query": c["SQ_INSTS_VALU"] * 64 / n, "lds_per_query": c["SQ_INSTS_LDS"] * 64 / n,
               "achieved_wave_instr_per_s": rate, "frac": rate / PEAK,
               # the kernel's VALU is integer work: at 4 cycles per wave64 instruction (the no-window
               # ablation's 351 us for ~100 VALU per query at 2^27 fits it) the ceiling is half
               "frac_of_4cycle_issue": rate / (PEAK / 2)}
        if tag == "27":
            lds = counters(SRC / "lds27_counters.csv")
            cyc = us * 1e-6 * 2.4e9
            rec["lds_bank_conflict_frac"] = lds["SQ_LDS_BANK_CONFLICT"] / 256 / cyc
            rec["wave_wait_dependency_frac"] = lds["SQ_WAIT_INST_ANY"] / lds["SQ_WAVE_CYCLES"]

        out[f"2^{tag}"] = rec
    dst = REPO / "profiles" / "query_valu.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
