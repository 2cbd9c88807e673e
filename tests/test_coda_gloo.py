"""Multi-rank CoDA orchestration on CPU (gloo, world 1/2/4/8) vs the reference trajectory.

World 8 runs BASELINE configs[2]'s averaging periods I = 1, 8, 32 (coda_w8_I*.npz, made by the
reference's own main.average_all over gloo at 8 ranks).

The product's CoDA loop, FlatState bookkeeping (segment table, count slots in the
all-reduced buffer, anchors, stage restarts) and its torch.distributed calls run
unchanged; only the kernels are served by the oracle (tests/cpu_kernels.py),
because this container has no GPU. The GPU variant of the same comparison,
through libdauc.so, is tests/test_coda_gpu.py.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch

import coda_parity
import cpu_kernels


def _load(golden, world, suffix=""):
    with np.load(golden / f"coda_w{world}{suffix}.npz") as z:
        return {k: z[k] for k in z.files}


def test_coda_world1_cpu_orchestration(golden, monkeypatch):
    cpu_kernels.install(monkeypatch)
    fx = _load(golden, 1)
    rec, coda = coda_parity.run_rank(fx, 0, 1, torch.device("cpu"))
    coda_parity.compare(fx, 0, rec)
    # stage-end averages (main.py:338-339) of the last stage
    w_avg_end = fx["r0_stage_w_avg_end"][-1]
    got = np.concatenate([coda.state.avg[o:o + n].numpy() for _, _, o, n in coda.state.entries])
    coda_parity.close(got, w_avg_end, "stage-end running average")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, golden_dir, q, suffix=""):
    import traceback
    from pathlib import Path

    import torch.distributed as dist

    try:
        torch.set_num_threads(1)
        cpu_kernels.install_in_process()
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        fx = _load(Path(golden_dir), world, suffix)
        rec, coda = coda_parity.run_rank(fx, rank, world, torch.device("cpu"))
        coda_parity.compare(fx, rank, rec)
        # BN buffers are local (main.py:35): ranks must still differ after averaging
        dist.destroy_process_group()
        q.put((rank, None))
    except BaseException:
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world,suffix", [(2, ""), (4, ""), (8, "_I1"), (8, "_I8_s4"), (8, "_I32_s4")])
@pytest.mark.timeout(300)
def test_coda_multirank_gloo(golden, world, suffix):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(golden), q, suffix)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    res = []
    while not q.empty():
        res.append(q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = [e for _, e in res if e]
    assert not errs, "\n".join(errs)
    assert sorted(r for r, _ in res) == list(range(world))
    fx = _load(golden, world, suffix)
    assert not np.allclose(fx["r0_bn"][-1], fx["r1_bn"][-1])  # reference keeps BN buffers local
    if world == 8:  # the period really varies the number of averaging rounds
        import json

        cfg = json.loads(str(fx["config"]))
        steps = len(fx["r0_t_total"])
        assert steps == (12 if cfg["numStages"] == 3 else 39) and steps // cfg["I"] >= 1
