"""bench.py's host logic (CPU): the launch contract and the configs[0] CPU baseline leg.

The N-rank GPU path itself is exercised on the GPU box (tests/test_bench_gpu.py); here only
what runs before any GPU call, and the gloo worker processes of the CPU baseline, which never
touch a GPU."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


def _bench():
    sys.path.insert(0, str(REPO))
    import bench

    return bench


def test_defaults_cover_the_baseline_configs():
    b = _bench()
    a = b.parse([])
    assert a.gpus == 1 and a.arch == "resnet50" and a.batch == 256 and a.I == 16  # configs[1]
    periods = [int(v) for v in a.sweep_I.split(",")]
    assert {1, 8, 32} <= set(periods)                                                 # configs[2]
    assert all(a.sweep_steps % I == 0 for I in periods)
    assert (a.auc_log2n, a.auc_pos) == (24, 0.01)                                     # configs[3]
    assert (a.auc2_log2n, a.auc2_pos) == (27, 0.001)                                  # configs[4]
    assert a.r18_steps > 0 and a.cpu_workers == 4                                     # configs[0]


def test_world_size_mismatch_fails_before_touching_the_gpu():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "4", "--no-train", "--no-auc",
                        "--no-surrogate", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=2" in r.stderr


def test_host_info_states_core_counts():
    h = _bench().host_info()
    assert h["nproc"] >= 1 and 1 <= h["cpu_budget"] <= h["affinity_cpus"]


@pytest.mark.parametrize("under_launcher", [False, True])
@pytest.mark.timeout(300)
def test_configs0_cpu_baseline_gloo_workers(monkeypatch, under_launcher):
    """configs[0]'s CPU path: gloo worker processes running the restated step with one
    average_all round (main.py:33-54) inside the timed window (small images to stay fast).
    under_launcher: called from rank 0 of a torch.distributed.run job (its env: the agent store,
    another job's MASTER_PORT and world size), as at N > 1 — the workers must form their own job."""
    if under_launcher:
        import socket

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            dead = s.getsockname()[1]
        for k, v in dict(TORCHELASTIC_USE_AGENT_STORE="True", TORCHELASTIC_RUN_ID="none", MASTER_ADDR="127.0.0.1",
                         MASTER_PORT=str(dead), RANK="0", WORLD_SIZE="8", LOCAL_RANK="0",
                         LOCAL_WORLD_SIZE="8").items():
            monkeypatch.setenv(k, v)
    b = _bench()
    args = b.parse(["--cpu-steps", "8", "--image-size", "32", "--cpu-workers", "2"])
    host = dict(b.host_info(), cpu_budget=2)
    r = b.cpu_baseline_configs0(args, host)
    assert "error" not in r, r
    assert r["workers"] == 2 and r["cores"] == 2 and r["value"] > 0
    assert r["params"] == 11_177_538 and r["params_finite"]
    assert r["averaging_round_ms"] > 0


def test_shipped_conv1x1_plans_load():
    """The shipped engine plan (measured once on MI355X) parses into fixed choices for the bench
    shapes, so no rank times engines at run time for them."""
    from distributedauc_amd import conv1x1 as C

    saved = dict(C.plans)
    try:
        C.plans.clear()
        C._load_plans()
        assert len(C.plans) >= 30
        key = (200704, 512, 128, __import__("torch").bfloat16, "dgrad_acc")  # ResNet-50 layer1 conv1 + skip
        assert key in C.plans
        assert all(v in ("gemm", "conv", "fconv") or v.startswith("gemm") for v in C.plans.values())
    finally:
        C.plans.clear()
        C.plans.update(saved)


def test_step_roofline_helpers():
    """the step's FLOP from the layer shapes (ResNet-50 b256 224^2: 4.09 GMAC per image
    forward; 3 x 2 MAC per step except the stem's input gradient) and the fused BN calls' bytes."""
    import ctypes

    import bench

    f = bench.backbone_flops("resnet50", 224, 256)
    assert abs(f["forward_gmac"] / 256 - 4.087) < 0.01
    stem = 256 * 112 * 112 * 64 * 3 * 49
    assert f["flop_per_step"] == 6 * int(f["forward_gmac"] * 1e9 + 0.5) - 2 * stem
    vp = ctypes.c_void_p
    M, C = 1000, 64
    act = M * C * 2
    # forward: x (stats) + x, residual, y (apply) + mask
    fwd = [vp(1), 2, M, C, vp(1), 1, vp(1), vp(1), vp(1), vp(1), 0.1, 1e-5, vp(1), vp(1), vp(1), vp(1), vp(1), 0, vp(1)]
    assert bench.bn_forward_bytes(fwd) == 4 * act + act // 16
    fwd[4], fwd[13] = vp(0), vp(0)  # no residual, no mask
    assert bench.bn_forward_bytes(fwd) == 3 * act
    # backward with the mask and a residual gradient: reduce dy + mask + x + dz, dx pass dz + x + dx
    bwd = [vp(1), vp(0), vp(1), vp(1), 2, M, C, 1, vp(1), vp(1), vp(1), vp(1), vp(1), vp(1), vp(1), vp(1), 0, vp(1)]
    assert bench.bn_backward_bytes(bwd) == (3 * act + act // 16) + 3 * act
    bwd[11] = vp(0)  # no residual: both passes read dy + mask + x, the second writes dx
    assert bench.bn_backward_bytes(bwd) == 2 * (2 * act + act // 16) + act


def test_cpu_baselines_at_one_gpu_only():
    """The bench contract times the CPU baselines on rank 0 at N = 1 only; --cpu-baseline-any-n
    keeps them for rehearsals, --no-cpu-baseline drops them everywhere."""
    b = _bench()
    assert b.cpu_baseline_on(b.parse([]), 1)
    assert not b.cpu_baseline_on(b.parse([]), 2)
    assert not b.cpu_baseline_on(b.parse([]), 8)
    assert b.cpu_baseline_on(b.parse(["--cpu-baseline-any-n"]), 8)
    assert not b.cpu_baseline_on(b.parse(["--no-cpu-baseline"]), 1)
    assert not b.cpu_baseline_on(b.parse(["--no-cpu-baseline", "--cpu-baseline-any-n"]), 4)
