"""Timeline of the surrogate chunk kernel (instrumented build, DAUC_SUR_X=9): per-block wall-clock stamps.

DAUC_LIB=tuning/libdauc_x_9.so python scripts/probe_sur_timeline.py
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np
import torch

from distributedauc_amd import _lib, ops

dev = torch.device("cuda", 0)
B = 1 << 26
g = torch.Generator(device=dev).manual_seed(1)
h = torch.rand(B, device=dev, generator=g)
y = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
ab = torch.tensor([0.1, -0.2, 0.3], device=dev)
p = torch.tensor([0.1], device=dev)
dh = torch.empty(B, device=dev)
g3 = torch.zeros(3, device=dev)
for _ in range(5):
    ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, grad3=g3)
torch.cuda.synchronize()
ws = [t for k, t in ops.workspaces._ws.items() if k[2] == "surrogate"][0]
nblocks = B // 8192
kpers = 256 + 2048 * 6 * 8
gs = max(256, (nblocks + 63) // 64)
ng = (nblocks + gs - 1) // gs
off = kpers + (nblocks * 4 + ng) * 6 * 8
st = ws[off: off + nblocks * 64].cpu().numpy().view(np.uint64).reshape(nblocks, 8).astype(np.int64)
t0 = st[:, 0].min()
rel = (st - t0) * 10 / 1000.0  # 100 MHz -> us
spin = [min(b * 1 + gs - 1, nblocks - 1) for b in range(0, nblocks, gs)]
out = {"kernel_span_us": float(rel[:, 2].max()), "last_block_start_us": float(rel[:, 0].max()),
       "data_end_p50_us": float(np.median(rel[:, 2])), "block_life_p50_us": float(np.median(rel[:, 2] - rel[:, 0])),
       "block_math_p50_us": float(np.median(rel[:, 1] - rel[:, 0])),
       "spinners": [{"blk": int(b), "start": float(rel[b, 0]), "data_end": float(rel[b, 2]), "l1_done": float(rel[b, 3]),
                     "l2_done": float(rel[b, 4]) if b == nblocks - 1 else None} for b in spin]}
print(json.dumps(out))
# dispatch order: correlation of start time with block index
order = np.argsort(rel[:, 0])
print(json.dumps({"start_vs_index_max_displacement": int(np.abs(order - np.arange(nblocks)).max()),
                  "start_first8": rel[:8, 0].tolist(), "end_max_block": int(rel[:, 2].argmax())}))
