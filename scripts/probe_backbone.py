"""Probe: ResNet fwd+bwd step time under different MIOpen / layout settings (one config per process)."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributedauc_amd.backbone import build_backbone

p = argparse.ArgumentParser()
p.add_argument("--layout", default="cl"); p.add_argument("--dtype", default="bf16")
p.add_argument("--benchmark", type=int, default=0); p.add_argument("--batch", type=int, default=256)
p.add_argument("--arch", default="resnet50"); p.add_argument("--size", type=int, default=224)
p.add_argument("--steps", type=int, default=5)
p.add_argument("--fused", type=int, default=0)
p.add_argument("--gemm1x1", type=int, default=0)
a = p.parse_args()
torch.backends.cudnn.benchmark = bool(a.benchmark)
dev = torch.device("cuda", 0)
net = build_backbone(a.arch).to(dev)
if a.fused:
    net.set_fused_bn(True)
if a.gemm1x1:
    net.set_gemm_conv1x1(True)
x = torch.randn(a.batch, 3, a.size, a.size, device=dev)
if a.layout == "cl":
    net = net.to(memory_format=torch.channels_last); x = x.contiguous(memory_format=torch.channels_last)
ctx = (lambda: torch.autocast("cuda", dtype=torch.bfloat16)) if a.dtype == "bf16" else (lambda: torch.autocast("cuda", enabled=False))
def step():
    with ctx():
        out = net(x)
    out[:, 1].sum().backward()
t0 = time.perf_counter()
for _ in range(2): step()
torch.cuda.synchronize(); t1 = time.perf_counter()
for _ in range(a.steps): step()
torch.cuda.synchronize(); t2 = time.perf_counter()
ms = (t2 - t1) / a.steps * 1e3
print(f"RESULT fused={a.fused} gemm1x1={a.gemm1x1} layout={a.layout} dtype={a.dtype} bench={a.benchmark} find={os.environ.get('MIOPEN_FIND_MODE','default')} "
      f"warm={t1-t0:.1f}s step={ms:.1f}ms imgs/s={a.batch/ms*1e3:.0f}", flush=True)
