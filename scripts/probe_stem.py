"""Micro-benchmark of the 7x7 stem kernels (csrc/conv_stem.hip) at ResNet-50 b256 against MIOpen's
(torch bf16 conv2d / convolution_backward): HIP-event time per call, one JSON line per op.

    python scripts/probe_stem.py [reps]
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributedauc_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn((256, 3, 224, 224), device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn((64, 3, 7, 7), device=dev, generator=g) / 12).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
dy = torch.randn((256, 64, 112, 112), device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = ops.stem_conv_forward(x, w)
dw = ops.stem_conv_wgrad(x, dy)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


flop = 2 * 256 * 112 * 112 * 64 * 147
hbm = {"fwd": 256 * 112 * 112 * 64 * 2 + x.numel() * 2, "wgrad": dy.numel() * 2 + x.numel() * 2}
rows = {
    "fwd": timed(lambda: ops.stem_conv_forward(x, w, out=y)),
    "wgrad": timed(lambda: ops.stem_conv_wgrad(x, dy, out=dw)),
    "miopen_fwd": timed(lambda: F.conv2d(x, w, stride=2, padding=3)),
    "miopen_wgrad": timed(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [3, 3], [1, 1], False,
                                                                      [0, 0], 1, [False, True, False])),
}
for k, us in rows.items():
    b = hbm["fwd" if "fwd" in k else "wgrad"]
    print(json.dumps({"op": k, "us_per_call": us, "tflops": flop / us / 1e6, "tb_s": b / us / 1e6}), flush=True)
