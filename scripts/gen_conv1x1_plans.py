"""Measure the 1x1-conv engine plan once for the bench shapes and write it as the shipped plan file.

Run with DAUC_CONV1X1_PLANS="" (no plan file: every shape is timed on first use, best of 3 HIP-event
timings per engine, conv1x1._choose) on an MI355X: a few CoDA steps of ResNet-50 b256 and ResNet-18
b32 (224^2, bf16 channels-last, the bench's own setup), then conv1x1.dump_plans(out)."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

from distributedauc_amd import conv1x1  # noqa: E402

out = sys.argv[1]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for arch, batch, I in (("resnet50", 256, 16), ("resnet18", 32, 8)):
    coda, it = bench.make_coda(arch, batch, 224, I, 0.1, 2, 1, 0, dev)
    for _ in range(3):
        x, y = next(it)
        coda.train_step(x, y)
    torch.cuda.synchronize()
    print(arch, "loss", float(coda.last_loss), "plans so far", len(conv1x1.plans), flush=True)
    del coda, it
conv1x1.dump_plans(out)
print("wrote", out)
