"""RCCL rehearsal on the one-GPU box: the nccl backend (= RCCL) has to run every
collective the driver's N > 1 bench issues before that run does. A FRESH child process under
torch.distributed.run --nproc-per-node 1 (nothing touches the GPU before its init_process_group,
as in an 8-rank launch) brings up a one-rank nccl group and drives, with the world > 1 branches
forced on: the ResNet-50 94 MB flat all-reduce + finalise, averaging rounds inside training steps,
the fp64 alpha all-reduce, the two-step sharded exact AUC's uint8 slot and int64 record gathers
at configs[3] and configs[4] sizes (counts vs the C oracle), the pair-count record gather, the
split evaluation's broadcasts and score all-gather, a barrier and a HIP-graph capture after the
communicator exists (bit-identical to eager, and the reference trajectory within 1e-5). The bench
runs the same group with `--gpus 1 --backend nccl` (test below)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _clean_env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


@pytest.mark.timeout(600)
def test_rccl_rehearsal_one_rank(tmp_path):
    out = tmp_path / "rehearsal.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(REPO / "tests" / "rccl_rehearsal.py"), str(out)]
    r = subprocess.run(cmd, env=_clean_env(), capture_output=True, text=True, timeout=560)
    keep = os.environ.get("DAUC_BENCH_RECORD_DIR")
    if keep:
        Path(keep).mkdir(parents=True, exist_ok=True)
        (Path(keep) / "rccl_rehearsal.log").write_text(r.stderr[-20000:])
    assert r.returncode == 0, r.stderr[-4000:]
    rec = json.loads(out.read_text())
    if keep:
        (Path(keep) / "rccl_rehearsal.json").write_text(json.dumps(rec, indent=1))
    assert rec["backend"] == "nccl" and rec["world"] == 1
    steps = {s["step"]: s for s in rec["steps"]}
    r50 = steps["coda_round_r50"]
    assert r50["payload_bytes"] > 94_000_000 and r50["params_equal"] and r50["counts_folded"] and r50["alpha_finite"]
    assert steps["train_steps_r50_I2"]["finite"]
    assert steps["alpha_sums_fp64"]["equal"]
    for k in ("auc_two_step_2^24", "auc_two_step_2^27"):
        assert steps[k]["mode"] == "sharded" and steps[k]["match"], steps[k]
    assert steps["auc_pairs_2^24"]["match"]
    assert steps["split_evaluation"]["split"] and steps["split_evaluation"]["finite"]
    assert "barrier" in steps
    g = steps["graph_after_comm"]
    assert g["captures"] >= 1 and g["graph_equals_eager"] and g["matches_reference"] is True, g


@pytest.mark.timeout(600)
def test_bench_nccl_one_rank(tmp_path):
    """bench.py --gpus 1 --backend nccl: the whole bench on a one-rank RCCL group (torch.distributed.run
    child, world > 1 code paths), reduced sizes: the line reports the nccl group and a coda_round."""
    cmd = [sys.executable, str(REPO / "bench.py"), "--gpus", "1", "--backend", "nccl",
           "--arch", "resnet18", "--batch", "32", "--image-size", "64", "--steps", "4", "--warmup", "2",
           "--sweep-I", "1,2", "--sweep-steps", "2", "--eval-images", "256", "--r18-steps", "8",
           "--auc-log2n", "20", "--auc2-log2n", "21", "--auc-reps", "1", "--auc-shard-min", "0",
           "--sur-log2b", "16", "--sur-reps", "5", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=_clean_env(), capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    keep = os.environ.get("DAUC_BENCH_RECORD_DIR")
    if keep:
        (Path(keep) / "bench_n1_nccl_rehearsal.json").write_text(lines[0] + "\n")
    assert out["n_gpus"] == 1 and out["process_group"]["backend"] == "nccl"
    assert out["process_group"]["world_size"] == 1
    assert out["coda_round"]["ms_per_round"] > 0 and out["coda_round"]["backend"] == "nccl"
    assert out["training_eval"]["method"] == "split"
    for k in ("auc_eval", "auc_eval_extreme"):
        assert out[k]["methods_agree"] and out[k]["sort_mode"] == "sharded"
    assert out["configs0"]["gpu"]["graph"]  # HIP-graph replay with the communicator up
