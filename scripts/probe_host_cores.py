"""The GPU box's host CPU share: nproc, the affinity mask, the cgroup CPU quota,
and the reference CPU path's ResNet-50 step (oracle restatement, torch CPU fp32) at several thread
counts, at batch 32 (a bounded sample). Never touches the GPU. Prints one JSON line."""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import torch  # noqa: E402


def cgroup_quota():
    for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = Path(f).read_text().split()
        except OSError:
            continue
        if f.endswith("cpu.max"):
            if txt[0] == "max":
                return {"file": f, "cpus": None, "raw": " ".join(txt)}
            return {"file": f, "cpus": int(txt[0]) / int(txt[1]), "raw": " ".join(txt)}
        q = int(txt[0])
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        return {"file": f, "cpus": None if q < 0 else q / per, "raw": f"{q} {per}"}
    return None


def step_time(threads, batch, arch="resnet50", size=224):
    from distributedauc_amd.backbone import build_backbone
    from oracle import reference_cpu as R

    torch.set_num_threads(threads)
    torch.manual_seed(0)
    net = build_backbone(arch, num_classes=2)
    a, b, al = (torch.zeros(1, requires_grad=True) for _ in range(3))
    p = torch.tensor([0.1])
    x = torch.randn(batch, 3, size, size)
    lab = torch.where(torch.rand(batch) < 0.1, 1, -1)
    ts = []
    for _ in range(2):
        t0 = time.perf_counter()
        loss = R.surrogate_loss(net(x)[:, 1], lab, a, b, al, p)
        net.zero_grad()
        loss.backward()
        ts.append(time.perf_counter() - t0)
    return ts


def main():
    aff = len(os.sched_getaffinity(0))
    rec = {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup": cgroup_quota(),
           "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "runs": []}
    print(json.dumps({k: v for k, v in rec.items() if k != "runs"}), file=sys.stderr, flush=True)
    for th in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "16,64,256").split(",")]:
        th = min(th, aff)
        ts = step_time(th, 32)
        rec["runs"].append({"threads": th, "batch": 32, "step_s": ts, "imgs_per_sec": 32 / ts[-1]})
        print(json.dumps(rec["runs"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
