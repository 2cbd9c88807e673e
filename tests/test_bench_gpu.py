"""bench.py launches its own ranks: ``--gpus 2`` without a launcher must measure 2 ranks.

On the one-GPU box the two ranks share cuda:0 over gloo (the RCCL backend needs one GPU per
rank and is refused with a clear error instead). The full N-rank RCCL runs are the driver's."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


@pytest.mark.timeout(600)
def test_bench_self_launches_two_ranks():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--backend", "gloo", "--no-train",
                        "--no-surrogate", "--no-cpu-baseline", "--auc-log2n", "18", "--auc2-log2n", "0",
                        "--auc-reps", "1"], env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-3000:]  # stdout carries the JSON record and nothing else
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["process_group"]["world_size"] == 2 and out["process_group"]["backend"] == "gloo"
    assert out["auc_eval"]["methods_agree"] and out["auc_eval"]["P"] > 0


@pytest.mark.timeout(300)
def test_bench_refuses_rccl_with_fewer_gpus_than_ranks():
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU: the RCCL path is the driver's multi-GPU run")
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--no-train", "--no-surrogate",
                        "--no-cpu-baseline", "--no-auc"], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode != 0
    assert "one GPU per rank" in r.stderr
