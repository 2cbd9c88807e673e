"""Where the one-launch loss spends its tail: the tuning build's stamped tail kernels at B = 2^26,
s_memrealtime stamps (100 MHz) read back from the workspace's stamp region (include/dauc_tuning.h):
variant 5 = the product's kernel (the last 64 workgroups reduce), 7 = the early-reducer kernel
(lag 4096). Per call: the time every workgroup stored its row, and per reducer the start /
own-group-done / [group totals added: final] / block-sum-done / publish / finalize times,
relative to the LAST row store of the call. One JSON line per call plus a summary.
    python scripts/probe_tail_stamps.py [calls] [variant]"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributedauc_amd import _lib, ops  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
B = 1 << 26
R = {5: 64, 14: 64, 21: 128}.get(variant, 256)  # group-total rows the kernel's workspace layout reserves
g = torch.Generator(device=dev).manual_seed(7)
h = torch.rand(B, device=dev, generator=g)
y = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
ab = torch.tensor([0.1, -0.2, 0.3], device=dev)
p = torch.tensor([0.1], device=dev)
dh = torch.empty(B, device=dev)
o = torch.zeros(6, dtype=torch.float64, device=dev)
L = _lib.tuning()
ws = ops.workspaces.get(dev, "surrogate_tuning", L.dauc_surrogate_workspace_size(B))
nb = B // 4096
chunk = nb * 48 + 256 + -(-nb // 512) * 48
off = 256 + 2048 * 48 + -(-chunk // 256) * 256  # surrogate.hip tail_offset
st0 = off + 256 + (nb + R) * 80                  # stamps after the header, rows and group totals
for _ in range(300):
    ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, out64=o, variant=0)
ref = o.clone()
recs = []
for c in range(calls):
    ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, out64=o, variant=variant)
    torch.cuda.synchronize()
    assert torch.allclose(o, ref, rtol=1e-12, atol=0), (o, ref)
    s = ws[st0: st0 + (nb + 8 * R) * 8].view(torch.int64).cpu().numpy().astype(np.float64) * 10.0 / 1e3  # us
    rows, red = s[:nb], s[nb:].reshape(R, 8)
    t_last, first = rows.max(), rows.min()
    used = red[:, 0] > 0
    fin = R - 1 if variant in (5, 14, 21) else int(np.flatnonzero(used).max())
    others = [i for i in np.flatnonzero(used) if i != fin]
    pub = red[others, 3] - t_last
    rec = {"call": c, "stream_us": t_last - first, "rows_last_1pct_us": float(t_last - np.percentile(rows, 99)),
           "reducers": int(used.sum()),
           "group_published_us": [float(pub.min()), float(np.median(pub)), float(pub.max())],
           "final_start_us": float(red[fin, 0] - t_last), "final_own_group_us": float(red[fin, 1] - t_last),
           "final_totals_us": float(red[fin, 4] - t_last), "final_sum_us": float(red[fin, 2] - t_last),
           "final_done_us": float(red[fin, 5] - t_last)}
    recs.append(rec)
    print(json.dumps(rec), flush=True)
keys = ["stream_us", "final_own_group_us", "final_totals_us", "final_sum_us", "final_done_us"]
print(json.dumps({"variant": variant, "summary": {k: float(np.median([r[k] for r in recs])) for k in keys},
                  "max_group_published_us": float(np.median([r["group_published_us"][2] for r in recs]))}))
