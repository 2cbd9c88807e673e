"""Tune the bench's hipBLASLt GEMMs with PyTorch TunableOp, every candidate solution checked
against the default one (numerical check), and write the selections as a CSV.

r01 found one hipBLASLt solution that returns wrong values on one ResNet-50 shape (DESIGN §6,
profiles/r02/tunableop/); the numerical check rejects such a solution at tuning time. Run on an
MI355X:  python scripts/tune_gemms.py <out.csv>  (a few CoDA steps of ResNet-50 b256, the
bench's own setup; the file is written when the process exits).
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.cuda.tunable as tunable  # noqa: E402

out = sys.argv[1]
tunable.enable(True)
tunable.tuning_enable(True)
tunable.set_numerical_check_tolerances(True, atol=1e-2, rtol=1e-2)
tunable.set_max_tuning_duration(40)
tunable.set_filename(out)

import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
coda, it = bench.make_coda("resnet50", 256, 224, 16, 0.1, 2, 1, 0, dev)
for _ in range(3):
    x, y = next(it)
    coda.train_step(x, y)
torch.cuda.synchronize()
print("loss", float(coda.last_loss), "tuned GEMMs", len(tunable.get_results()), flush=True)
