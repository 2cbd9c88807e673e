"""A/B of the loss kernel variants at B = 2^26 (tuning build, include/dauc_tuning.h), HIP events
around `reps` back-to-back calls per variant, variants interleaved, `rounds` rounds.
    python scripts/ab_surrogate.py [rounds] [reps] [variants comma-separated]"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import ops  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
variants = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,3,20,22").split(",")]
dev = torch.device("cuda", 0)
B = 1 << 26
g = torch.Generator(device=dev).manual_seed(7)
h = torch.rand(B, device=dev, generator=g)
y = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
ab = torch.tensor([0.1, -0.2, 0.3], device=dev)
p = torch.tensor([0.1], device=dev)
dh = torch.empty(B, device=dev)
o = torch.zeros(6, dtype=torch.float64, device=dev)
ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, out64=o, variant=0)
ref, dh_ref = o.clone(), dh.clone()
for v in variants:
    for _ in range(400):
        ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, out64=o, variant=v)
    torch.cuda.synchronize()
    if v not in (3, 4):  # 3 / 4 reduce nothing
        # other row groupings add the same fp64 partials in another order: equal to ~1e-13
        assert torch.allclose(o, ref, rtol=1e-12, atol=0), (v, o, ref)
        assert torch.equal(dh, dh_ref), v
torch.cuda.synchronize()
for r in range(rounds):
    for v in variants:
        for _ in range(50):
            ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, out64=o, variant=v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, out64=o, variant=v)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print(json.dumps({"round": r, "variant": v, "us": us, "frac": 9 * B / (us * 1e-6) / 8e12}), flush=True)
