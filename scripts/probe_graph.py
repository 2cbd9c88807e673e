"""Probe: is the ResNet-50 CoDA step (bench.py's configs[1] workload) host-issue-bound, and
does capturing one step body (a1-a5: label map, forward, surrogate, backward, pd_update,
zero_grad) in a HIP graph remove the idle gaps the rocprof trace shows at every step start?

Prints JSON lines: eager host-issue ms/step, eager wall ms/step, graph wall ms/step, and the
max |difference| of the flat parameters between an eager and a graphed run from the same
state (bf16 MIOpen split-K convolutions are not bitwise deterministic, so this is a tolerance
check, not parity).
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributedauc_amd.backbone import build_backbone  # noqa: E402
from distributedauc_amd.coda import CoDA  # noqa: E402
from distributedauc_amd.loader import DeviceLoader, SyntheticImageNet, imagenet_like_labels  # noqa: E402


def main():
    steps = int(os.environ.get("STEPS", "20"))
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    split = 499
    labels = imagenet_like_labels(1 << 16, 1000, split, pos_ratio=0.1, seed=123)
    ds = SyntheticImageNet(labels, 224, split)
    loader = DeviceLoader(ds, np.arange(len(labels)), 256, dev, seed=1234, channels_last=True, pool=4)
    net = build_backbone("resnet50", num_classes=2).to(dev).to(memory_format=torch.channels_last)
    net.set_fused_bn(True).set_gemm_conv1x1(True)
    coda = CoDA(net, lr=0.1, gamma=2000.0, T0=10 ** 9, I=16, split_index=split, world=1, rank=0,
                autocast_dtype=torch.bfloat16, device=dev)
    it = iter(loader)
    coda.average_all()
    coda.begin_stage(1, it)
    for _ in range(5):
        x, y = next(it)
        coda.train_step(x, y)
    torch.cuda.synchronize()

    # eager: host issue time vs wall time
    t0 = time.perf_counter()
    host = []
    for _ in range(steps):
        x, y = next(it)
        h0 = time.perf_counter()
        coda.train_step(x, y)
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"eager_host_issue_ms_per_step": 1e3 * float(np.mean(host)),
                      "eager_host_issue_p50_ms": 1e3 * float(np.median(host)),
                      "eager_issue_loop_ms_per_step": 1e3 * (t1 - t0) / steps,
                      "eager_wall_ms_per_step": 1e3 * (t2 - t0) / steps}), flush=True)

    # graph capture of the step body
    st = coda.state
    xs, ys = next(it)
    xs, ys = xs.clone(), ys.clone()
    snap = st.flat.clone(), st.avg.clone(), st.lcounts.clone(), st.gcounts.clone()

    def body():
        return coda.step_body(xs, ys)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    torch.cuda.synchronize()
    print(json.dumps({"captured": True}), flush=True)

    def restore():
        st.flat.copy_(snap[0]); st.avg.copy_(snap[1]); st.lcounts.copy_(snap[2]); st.gcounts.copy_(snap[3])

    # same state, same input: eager vs graph after 4 steps
    restore()
    for _ in range(4):
        body()
    eager = st.flat.clone()
    restore()
    for _ in range(4):
        g.replay()
    graphed = st.flat.clone()
    d = (eager - graphed).abs()
    print(json.dumps({"max_abs_diff_eager_vs_graph": float(d.max()),
                      "max_abs_flat": float(eager.abs().max()),
                      "frac_bit_equal": float((eager == graphed).float().mean())}), flush=True)

    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        x, y = next(it)
        xs.copy_(x)
        ys.copy_(y)
        if (k + 1) % 16 == 0:
            coda.average_all()
        g.replay()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"graph_wall_ms_per_step": 1e3 * (t2 - t0) / steps,
                      "graph_imgs_per_s": 256 * steps / (t2 - t0)}), flush=True)


if __name__ == "__main__":
    main()
