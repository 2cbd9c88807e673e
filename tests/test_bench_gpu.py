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


@pytest.mark.timeout(900)
def test_bench_full_two_ranks_gloo(tmp_path):
    """Every leg the driver's N > 1 run takes, at reduced sizes, as 2 gloo ranks on cuda:0 (VERDICT
    r03 #2): training + the period sweep, coda_round, the split in-training evaluation, the
    configs[0] GPU leg, both exact-AUC legs (sharded sort method and pair count), the loss kernel
    leg and (--cpu-baseline-any-n: the contract times them at N = 1 only) the CPU baselines. One JSON
    line on stdout, world size 2."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--arch", "resnet18", "--batch", "32", "--image-size", "64", "--steps", "4", "--warmup", "2",
           "--sweep-I", "1,2", "--sweep-steps", "2", "--eval-images", "256", "--r18-steps", "8",
           "--auc-log2n", "20", "--auc2-log2n", "21", "--auc-reps", "1", "--auc-shard-min", "0", "--sur-log2b", "16", "--sur-reps", "5",
           "--cpu-workers", "2", "--cpu-steps", "2", "--cpu-sklearn-full", "0", "--cpu-max-s", "20",
           "--cpu-baseline-any-n"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=840)
    (tmp_path / "stderr.log").write_text(r.stderr)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    out_dir = os.environ.get("DAUC_BENCH_RECORD_DIR")
    if out_dir:  # the GPU runner keeps the line (profiles/r04/)
        Path(out_dir).mkdir(parents=True, exist_ok=True)
        (Path(out_dir) / "bench_n2_gloo_full.json").write_text(lines[0] + "\n")
    assert out["n_gpus"] == 2 and out["process_group"]["world_size"] == 2
    assert out["value"] > 0 and out["config"]["parallelism"] == "dp2"
    assert out["coda_round"]["ms_per_round"] > 0
    te = out["training_eval"]
    assert te["method"] == "split" and 0.0 <= te["auc"] <= 1.0 and "auc_rank0_scoring" in te
    assert [rec["I"] for rec in out["period_sweep"]["records"]] == [1, 2]
    for k in ("auc_eval", "auc_eval_extreme"):
        assert out[k]["methods_agree"] and out[k]["sort_mode"] == "sharded"
    assert out["auc_eval_extreme"]["cpu_baseline"]["oracle_counts"]["match"]
    assert out["configs0"]["gpu"]["n_gpus"] == 2 and out["configs0"]["cpu"]["params_finite"]
    assert out["surrogate_kernel"]["roofline"]["achieved"] > 0
    assert out["cpu_baseline"]["value"] > 0


@pytest.mark.timeout(600)
def test_bench_default_sizes_two_ranks_gloo(tmp_path):
    """the driver's N > 1 bench at the BASELINE sizes -- ResNet-50 b256 224^2 bf16 at
    I = 16 with the HIP backbone kernels, the period sweep with real averaging rounds, configs[3]
    (2^24 @ 1 %) and configs[4] (2^27 @ 0.1 %) sharded over the ranks -- as 2 gloo ranks on cuda:0.
    Fewer steps than the driver's so the test stays short; every leg and every size is the default
    one, and, as in the driver's N > 1 runs, no CPU baseline (timed at N = 1 only)."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "4", "--warmup", "3",
           "--sweep-I", "1,8,16", "--sweep-steps", "16", "--eval-images", "1024", "--r18-steps", "8", "--auc-reps", "1",
           "--sur-reps", "10"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=560)
    (tmp_path / "stderr.log").write_text(r.stderr)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    out_dir = os.environ.get("DAUC_BENCH_RECORD_DIR")
    if out_dir:
        Path(out_dir).mkdir(parents=True, exist_ok=True)
        (Path(out_dir) / "bench_n2_gloo_default_sizes.json").write_text(lines[0] + "\n")
    assert out["n_gpus"] == 2 and out["process_group"]["world_size"] == 2
    assert out["config"]["global_batch"] == 512 and out["config"]["image_size"] == 224 and out["config"]["I"] == 16
    assert out["config"]["params"] == 23_512_130 and out["value"] > 0
    assert out["coda_round"]["payload_bytes"] == 94_048_788 and out["coda_round"]["ms_per_round"] > 0
    assert [rec["I"] for rec in out["period_sweep"]["records"]] == [1, 8, 16]
    for k, P in (("auc_eval", 168478), ("auc_eval_extreme", 134447)):
        assert out[k]["methods_agree"] and out[k]["sort_mode"] == "sharded", k
        assert out[k]["P"] == P  # the bench's synthetic_scores at 2^24 @ 1 % and 2^27 @ 0.1 %
    assert out["step_roofline"]["flop_per_step"] > 6e12 and out["step_roofline"]["bn"]["bytes_per_step"] > 0
    assert out["cpu_baseline"] is None and "N = 1 only" in out["cpu_baseline_note"]


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
