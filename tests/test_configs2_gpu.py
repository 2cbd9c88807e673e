"""BASELINE configs[2]: ResNet-50 CoDA over 8 ranks, averaging of (w, a, b, alpha) at I in {1, 8, 32}.

The real workload (ResNet-50, batch 256 per rank, 224^2, bf16 autocast backbone, fp32 master
weights: 161 parameter tensors, 23,512,130 parameters) runs as 8 gloo ranks sharing cuda:0 — the
only multi-rank form one GPU box allows; the averaging itself is the same code the RCCL run uses
(CoDA.average_all: ONE all-reduce of flat[:n_reduce] + dauc_coda_finalize, main.py:33-54). Every
rank is built by bench.make_coda, as the bench does (same seeds, per-rank data shards).

Schedule (main.py:289-301: a round fires at the start of step t when t % I == 0, before its forward):
  I = 1   steps 1-2          -> 2 rounds
  I = 8   steps 1-8          -> 1 round (step 8)
  I = 32  steps 29-32        -> 1 round (step 32; the step counter is advanced to 28 first, so the
                                window holds the round without 28 unchecked steps in front of it)

Checked on every step of every rank: the 161-segment pd_update launch bit-exact against the C oracle
over all 23.5 M parameters, and a, b, alpha against the oracle's scalar update (tests/update_check.py).
Checked at every round:
  * flat[:n_reduce] after the round is bit-identical on all 8 ranks (rank 0's is broadcast and
    compared with torch.equal);
  * the averaged parameters, a, b, alpha equal the fp64 mean of the 8 gathered pre-round buffers
    within fp32 sum-order tolerance: |avg - mean64| <= 2^-20 * mean_r |x_r| + 2^-126 per element
    (a sum of 8 fp32 values in any order carries at most 7 roundings of <= 2^-24 relative to the
    running magnitudes, plus one for the division);
  * the class counts exact: gpos, gneg (fp32) equal the positives / negatives drawn by all ranks
    in every completed step, and each rank's local counts are zero.
"""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]
WORLD = 8
PLAN = ((1, 0, 2), (8, 0, 8), (32, 28, 4))  # (I, t_total before the window, steps)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, errq, progress):
    import torch
    import torch.distributed as dist

    sys.path[:0] = [str(REPO), str(REPO / "tests")]
    try:
        import bench
        import update_check

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)

        def note(msg):
            if rank == 0 and progress:
                with open(progress, "a") as f:
                    f.write(msg + "\n")

        coda, it = bench.make_coda("resnet50", 256, 224, PLAN[0][0], 0.1, 2, world, rank, dev)
        st = coda.state
        assert len(st.entries) == 161 and st.numel() == 23_512_130
        checks = update_check.install(coda, f"rank {rank}")
        drawn = torch.zeros(2, dtype=torch.float64)  # positives, negatives of this rank's completed steps
        rounds = {"n": 0}
        orig_average = coda.average_all

        def checked_average():
            torch.cuda.synchronize()
            pre = st.flat[: st.n_reduce].cpu()
            gathered = [torch.empty_like(pre) for _ in range(world)] if rank == 0 else None
            dist.gather(pre, gathered, dst=0)
            orig_average()
            torch.cuda.synchronize()
            post = st.flat[: st.n_reduce].cpu()
            ref = post.clone()
            dist.broadcast(ref, src=0)
            assert torch.equal(post, ref), f"rank {rank}: flat differs from rank 0 after round {rounds['n']}"
            if rank == 0:
                x = torch.stack(gathered)[:, : st.n_avg].double()
                mean = x.mean(0)
                tol = 2.0 ** -20 * x.abs().mean(0) + 2.0 ** -126
                err = (post[: st.n_avg].double() - mean).abs()
                bad = int((err > tol).sum())
                assert bad == 0, f"round {rounds['n']}: {bad} elements off the fp64 mean (max err {float(err.max())})"
            tot = drawn.clone()
            dist.all_reduce(tot)
            g = st.gcounts.cpu().double()
            assert torch.equal(g, tot), f"rank {rank}: global counts {g.tolist()} != drawn {tot.tolist()}"
            assert st.lcounts.cpu().tolist() == [0.0, 0.0]
            rounds["n"] += 1
            note(f"round {rounds['n']} ok (I={coda.I}, t={coda.t_total})")

        coda.average_all = checked_average
        steps = 0
        for I, t0, n in PLAN:
            coda.I = I
            coda.t_total = t0
            for _ in range(n):
                x, labels = next(it)
                loss = coda.train_step(x, labels)
                assert torch.isfinite(loss).item()
                drawn += torch.tensor([float((labels > 499).sum()), float((labels <= 499).sum())], dtype=torch.float64)
                steps += 1
                note(f"step {steps} ok (I={I}, t={coda.t_total})")
        torch.cuda.synchronize()
        assert checks["updates"] == steps == sum(p[2] for p in PLAN)
        assert rounds["n"] == 4, rounds
        dist.barrier()
        dist.destroy_process_group()
        errq.put((rank, None))
    except BaseException as e:  # report to the parent
        import traceback

        errq.put((rank, traceback.format_exc()))
        raise SystemExit(1) from e


@pytest.mark.timeout(900)
def test_configs2_resnet50_8ranks_period_sweep(dev):
    """configs[2]'s workload at world 8 (gloo ranks on cuda:0), I = 1, 8, 32: rounds bit-identical
    across ranks and equal to the fp64 mean, counts exact, every update bit-exact vs the oracle."""
    import torch.multiprocessing as mp

    out = REPO / "gpurun_out"
    progress = str(out / "configs2_progress.log") if out.is_dir() else ""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q, progress)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(840)
    errs = []
    while not q.empty():
        errs.append(q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    bad = [e for _, e in errs if e]
    assert not bad, "\n".join(bad)
    assert len(errs) == WORLD and all(p.exitcode == 0 for p in procs)
