"""Times the fused BN forward (stats + apply, ReLU mask) and backward (reduce + dx, from the mask;
with and without the residual gradient) at the ResNet-50 b256 layer shapes through the C ABI, one
JSON line per shape. The row-block walk follows DAUC_BN_INTERLEAVE / DAUC_BN_ROWBLOCKS (read once
per process), so A/B runs are separate processes.

  python scripts/probe_bn.py [--reps 30] [--tag name]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(256, 64, 112, 112), (256, 64, 56, 56), (256, 256, 56, 56), (256, 128, 28, 28), (256, 512, 28, 28),
          (256, 256, 14, 14), (256, 1024, 14, 14), (256, 512, 7, 7), (256, 2048, 7, 7)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    from distributedauc_amd import _lib
    from distributedauc_amd.ops import _ptr, _stream, check, workspaces

    dev = torch.device("cuda:0")
    L = _lib.load()
    st = _stream(dev)
    for (N, C, H, W) in SHAPES:
        M = N * H * W
        g = torch.Generator(device=dev).manual_seed(C + H)
        x = torch.randn(N, C, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn_like(x).contiguous(memory_format=torch.channels_last)
        y, dx, dres = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
        mask = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
        gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        mean, invstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
        dgamma, dbeta = torch.empty(C, device=dev), torch.empty(C, device=dev)
        ws = workspaces.get(dev, "bn_probe", L.dauc_bn_workspace_size(M, C))

        def fwd():
            check(L.dauc_bn_act_forward(_ptr(x), 2, M, C, None, 1, _ptr(gamma), _ptr(beta), None, None, 0.1, 1e-5,
                                        _ptr(y), _ptr(mask), _ptr(mean), _ptr(invstd), _ptr(ws), ws.numel(), st),
                  "forward")

        def bwd(res):
            check(L.dauc_bn_act_backward(_ptr(dy), None, _ptr(mask), _ptr(x), 2, M, C, 1, _ptr(gamma), _ptr(mean),
                                         _ptr(invstd), _ptr(dres) if res else None, _ptr(dx), _ptr(dgamma),
                                         _ptr(dbeta), _ptr(ws), ws.numel(), st), "backward")

        out = {"tag": a.tag, "shape": [N, C, H, W], "M": M,
               "interleave": os.environ.get("DAUC_BN_INTERLEAVE", "0")}
        for name, fn in (("fwd", fwd), ("bwd", lambda: bwd(False)), ("bwd_res", lambda: bwd(True))):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            out[name + "_us"] = round(e0.elapsed_time(e1) * 1000.0 / a.reps, 2)
        out["mean_sum"] = float(mean.double().sum())
        out["dgamma_sum"] = float(dgamma.double().sum())
        print(json.dumps(out), flush=True)
        del x, dy, y, dx, dres, mask
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
