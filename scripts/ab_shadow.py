"""A/B of the weight shadow's buffer sets on the headline step (round 6, ADVICE r05: two buffer sets
so that two forwards may precede one backward): ResNet-50 b256 224^2 bf16 CoDA steps (bench.make_coda,
the bench's switches) timed with the product's alternating two sets, and with refresh() pinned to one
set (the round-5 behaviour), interleaved. One JSON line per window. python scripts/ab_shadow.py [steps] [rounds]"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (sets the tuned MIOpen db)
import torch  # noqa: E402

from distributedauc_amd import backbone  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
bench.gemm_selections(os.path.join(bench.REPO, "distributedauc_amd", "tunableop_gfx950.csv"))
coda, it = bench.make_coda("resnet50", 256, 224, 16, 0.1, 4, 1, 0, dev, lr=0.01, flip=0.2, weight_shadow=3)
orig = backbone.WeightShadow.refresh


def pinned(self, flips=True):
    self._cur = 1  # refresh() flips it back to 0: always the first set
    orig(self, flips)


for _ in range(5):
    coda.train_step(*next(it))
for r in range(rounds):
    for name, fn in (("two_sets", orig), ("one_set", pinned)):
        backbone.WeightShadow.refresh = fn
        for _ in range(2):
            coda.train_step(*next(it))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            coda.train_step(*next(it))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"round": r, "form": name, "ms_per_step": dt / steps * 1e3, "imgs_per_sec": 256 * steps / dt}),
              flush=True)
backbone.WeightShadow.refresh = orig
