"""Is the evaluation forward bitwise repeatable within one process? ResNet-18 (channels_last, fused
BN, 1x1 GEMMs, bf16 autocast, eval mode) scores the same 4 batches of [48, 3, 32, 32] three times;
forward hooks keep every leaf module's output, and the first module whose output differs between
repetitions is printed per batch (the split-scoring test of main.Evaluator needs the bits of a
batch not to depend on what ran before it).
    python scripts/probe_eval_determinism.py [batch]"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedauc_amd import use_tuned_miopen_db  # noqa: E402
from distributedauc_amd.backbone import build_backbone  # noqa: E402
from distributedauc_amd.conv1x1 import fixed_engine  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 48
mode = sys.argv[2] if len(sys.argv) > 2 else "default"
if mode == "det":
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
elif mode == "algos":
    torch.use_deterministic_algorithms(True, warn_only=True)
print(json.dumps({"mode": mode}), flush=True)
use_tuned_miopen_db()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = build_backbone("resnet18", num_classes=2, head="softmax").to(dev).to(memory_format=torch.channels_last)
net.set_fused_bn(1).set_gemm_conv1x1(1)
xs = [torch.randn(bs, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last) for _ in range(4)]
acts: list = []  # per forward: [(module name, output)] in call order


def hook(name):
    def f(m, i, o):
        if acts:
            acts[-1].append((name, o.detach().clone() if torch.is_tensor(o) else None))
    return f


for n, m in net.named_modules():
    if len(list(m.children())) == 0:
        m.register_forward_hook(hook(n))
# a few training-mode forwards first (batch 16, as main.train's steps), then eval
with torch.autocast("cuda", dtype=torch.bfloat16):
    for _ in range(2):
        net(torch.randn(16, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)).sum().backward()
net.eval()
reps = 3
with torch.no_grad(), fixed_engine("gemm"), torch.autocast("cuda", dtype=torch.bfloat16):
    for r in range(reps):
        for x in xs:
            acts.append([])
            net(x)
torch.cuda.synchronize()
for b in range(len(xs)):
    for r in range(1, reps):
        first = None
        for (n, a), (_, c) in zip(acts[b], acts[r * len(xs) + b]):
            if a is None or c is None:
                continue
            if not torch.equal(a, c):
                first = {"module": n, "type": type(dict(net.named_modules())[n]).__name__,
                         "ndiff": int((a != c).sum()), "max": float((a.float() - c.float()).abs().max())}
                break
        print(json.dumps({"batch": b, "rep": r, "first_diff": first}), flush=True)
