"""Streaming ceiling for the surrogate's 5:4 read:write mix (tuning probe, not product code).

Usage:  python scripts/probe_stream.py --build        (here, on the CPU host: hipcc only)
        python scripts/probe_stream.py [--log2n 26]   (on the GPU box)
Prints one JSON line per kernel kind: µs per launch and GB/s of algorithmic bytes
(copy: 8 B/element, mix: 9 B/element).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "probe_stream.hip"
LIB = HERE / "libprobe_stream.so"
KINDS = {0: "copy S8", 1: "chunk S8 nt", 2: "chunk S16 nt", 3: "chunk S8 plain", 4: "chunk S8 ntload",
         5: "stride S4 2/CU", 6: "stride S8 1/CU", 7: "wide S2", 8: "wide S4", 9: "chunk S4 nt",
         10: "stride S8 4/CU", 11: "copy S16", 12: "pipe contig S8 2/CU", 13: "pipe contig S8 4/CU",
         14: "pipe stride S8 2/CU", 15: "pipe stride S8 4/CU", 16: "pipe stride S4 4/CU", 17: "pipe queue S8 2/CU",
         18: "pipe queue S8 4/CU", 19: "pipe queue S4 4/CU"}


def build() -> None:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    str(SRC), "-o", str(LIB)], check=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--log2n", type=int, default=26)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--kinds", default=None)
    a = ap.parse_args()
    if a.build:
        build()
        return
    import torch

    lib = ctypes.CDLL(str(LIB))
    lib.probe_run.restype = ctypes.c_float
    lib.probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                              ctypes.c_void_p, ctypes.c_int]
    n = 1 << a.log2n
    dev = torch.device("cuda", 0)
    h = torch.rand(n, device=dev)
    y = torch.where(torch.rand(n, device=dev) < 0.1, 1, -1).to(torch.int8)
    dh = torch.empty(n, device=dev)
    sink = torch.zeros(4, device=dev)
    torch.cuda.synchronize()
    kinds = [int(k) for k in a.kinds.split(",")] if a.kinds else list(KINDS)
    for rnd in range(2):
        for k in kinds:
            name = KINDS[k]
            ms = lib.probe_run(k, h.data_ptr(), y.data_ptr(), dh.data_ptr(), n, sink.data_ptr(), a.reps)
            bpe = 8 if name.startswith("copy") else 9
            print(json.dumps({"probe": name, "kind": k, "round": rnd, "n": n, "us": ms * 1e3,
                              "GBps": bpe * n / (ms * 1e-3) / 1e9 if ms > 0 else None}), flush=True)


if __name__ == "__main__":
    main()
