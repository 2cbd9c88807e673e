"""VALU-issue roofline of the labeled query kernel from committed rocprofv3 data.

Inputs (profiles/r02/pmc_query/): SQ_INSTS_VALU / SQ_INSTS_LDS per dispatch (one --pmc pass,
scripts/gpu_pmc_query_valu.sh) and the kernel's average duration from a separate
--kernel-trace --stats pass over the same command; LDS bank-conflict and wait counters
(scripts/gpu_pmc_query_lds.sh). Peak: 256 CUs x 4 SIMD-32 x 2.4 GHz / 2 cycles per wave64 VALU
instruction = 1.2288e12 wave-instructions/s (MI355X_MICROARCH.md, execution model).
Writes profiles/query_valu.json, which bench.py attaches to the AUC records."""
from __future__ import annotations

import collections
import csv
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
SRC = REPO / "profiles" / "r02" / "pmc_query"
PEAK = 256 * 4 * 2.4e9 / 2


def counters(f):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "query_labeled" in r["Kernel_Name"]:
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    vals = list(agg.values())
    return {k: sum(v[k] for v in vals) / len(vals) for k in vals[0]}


def avg_us(f):
    for r in csv.DictReader(open(f)):
        if "query_labeled" in r["Name"]:
            return float(r["AverageNs"]) / 1e3
    raise SystemExit(f"no query kernel in {f}")


def main():
    out = {"method": __doc__.split("\n\n")[1].replace("\n", " "), "peak_wave_instr_per_s": PEAK}
    for tag, n in (("27", 1 << 27), ("24", 1 << 24)):
        c = counters(SRC / f"valu{tag}_counters.csv")
        us = avg_us(SRC / f"trace{tag}_kernel_stats.csv")
        rate = c["SQ_INSTS_VALU"] / (us * 1e-6)
        rec = {"queries": n, "avg_launch_us": us, "valu_wave_instr": c["SQ_INSTS_VALU"],
               "valu_per_query": c["SQ_INSTS_VALU"] * 64 / n, "lds_per_query": c["SQ_INSTS_LDS"] * 64 / n,
               "achieved_wave_instr_per_s": rate, "frac": rate / PEAK}
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
