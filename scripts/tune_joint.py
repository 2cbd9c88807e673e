"""Re-measure the 1x1 engine plan with TunableOp's checked GEMM selections in the loop: every
(shape, direction) timed again (DAUC_CONV1X1_PLANS="" must be set by the caller) while TunableOp
tunes each new GEMM shape (numerical check against the default solution). Writes the plan and the
TunableOp CSV (at exit).   python scripts/tune_joint.py <plan.json> <tunableop.csv>
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.cuda.tunable as tunable  # noqa: E402

plan_out, csv_out = sys.argv[1], sys.argv[2]
tunable.enable(True)
tunable.tuning_enable(True)
tunable.set_numerical_check_tolerances(True, atol=1e-2, rtol=1e-2)
tunable.set_max_tuning_duration(40)
tunable.set_filename(csv_out)

import bench  # noqa: E402

from distributedauc_amd import conv1x1  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for arch, batch, I in (("resnet50", 256, 16), ("resnet18", 32, 8)):
    coda, it = bench.make_coda(arch, batch, 224, I, 0.1, 2, 1, 0, dev)
    for _ in range(3):
        x, y = next(it)
        coda.train_step(x, y)
    torch.cuda.synchronize()
    print(arch, "loss", float(coda.last_loss), "plans", len(conv1x1.plans), "tuned", len(tunable.get_results()),
          flush=True)
    del coda, it
conv1x1.dump_plans(plan_out)
print("wrote", plan_out)
