"""Micro-benchmark of the 3x3 weight-gradient kernel (csrc/conv_wgrad.hip) at the ResNet-50 b256
shapes, for kernel traces and PMC passes: each shape's call repeated `reps` times, HIP-event time per
call printed as one JSON line per shape.

    python scripts/probe_wgrad.py [reps] [form]

form (tuning build's dauc_set_wgrad_form): 1 gather, 2 / 3 window with 64- / 128-pixel chunks.
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import _lib, ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
if len(sys.argv) > 2:
    ops.set_wgrad_form(int(sys.argv[2]))
    _ctx = _lib.using(_lib.tuning())  # held for the whole run: its exit restores the product build
    _ctx.__enter__()
dev = torch.device("cuda", 0)
for C, H, stride in ((64, 56, 1), (128, 28, 1), (256, 14, 1), (512, 7, 1), (128, 56, 2), (256, 28, 2), (512, 14, 2)):
    g = torch.Generator(device=dev).manual_seed(C + H)
    x = torch.randn((256, C, H, H), device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H - 1) // stride + 1
    dy = torch.randn((256, C, Ho, Ho), device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = ops.conv3x3_wgrad(x, dy, stride)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.conv3x3_wgrad(x, dy, stride, out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    flop = 2 * 256 * Ho * Ho * C * 9 * C
    print(json.dumps({"form": sys.argv[2] if len(sys.argv) > 2 else "auto", "C": C, "H": H, "stride": stride, "us_per_call": us, "tflops": flop / us / 1e6}), flush=True)
