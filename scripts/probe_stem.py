"""Probe: the ResNet stem conv (7x7/2, 3 -> 64, pad 3) forward + weight gradient at batch 256,
channels-last bf16, as MIOpen sees it with C = 3, zero-padded C = 4 / 8, and as an im2col GEMM.

    python scripts/probe_stem.py
"""
from __future__ import annotations

import json

import torch
import torch.nn.functional as F


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    N = 256
    x3 = torch.randn(N, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w3 = (torch.randn(64, 3, 7, 7, device=dev) * 0.05).to(torch.bfloat16)
    gy = torch.randn(N, 64, 112, 112, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = []
    for C in (3, 4, 8):
        x = torch.zeros(N, C, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x[:, :3] = x3
        w = torch.zeros(64, C, 7, 7, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w[:, :3] = w3
        fwd = timed(lambda: F.conv2d(x, w, stride=2, padding=3))
        wrw = timed(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0],
                                                                1, [False, True, False]))
        y = F.conv2d(x, w, stride=2, padding=3)
        y3 = F.conv2d(x3, w3, stride=2, padding=3)
        out.append({"C": C, "fwd_us": fwd, "wgrad_us": wrw, "max_abs_diff_vs_C3": float((y - y3).abs().max())})
        print(json.dumps(out[-1]), flush=True)
    # im2col (unfold) + GEMM, K = 147 padded to 152
    def im2col():
        xp = F.pad(x3, (3, 3, 3, 3))
        cols = xp.unfold(2, 7, 2).unfold(3, 7, 2)  # N, C, 112, 112, 7, 7
        return cols.permute(0, 2, 3, 1, 4, 5).reshape(N * 112 * 112, 147)
    cols = im2col().contiguous()
    w2 = w3.reshape(64, 147)
    t_cols = timed(lambda: im2col().contiguous())
    t_mm = timed(lambda: torch.mm(cols, w2.t()))
    g2 = gy.permute(0, 2, 3, 1).reshape(-1, 64)
    t_wg = timed(lambda: torch.bmm(g2.view(32, -1, 64).transpose(1, 2), cols.view(32, -1, 147),
                                   out_dtype=torch.float32).sum(0))
    print(json.dumps({"im2col_torch_us": t_cols, "gemm_fwd_us": t_mm, "gemm_wgrad_split32_us": t_wg}), flush=True)


if __name__ == "__main__":
    main()
