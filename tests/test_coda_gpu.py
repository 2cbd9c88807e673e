"""One full CoDA run (2 stages, averaging every I=2 steps) on the GPU vs the reference trajectory.

The reference ran main.dppd_sg / main.average_all (gloo) / the inline loss on
TinyNet with these exact batches (tests/golden/make_golden.py). Here the same
schedule runs through libdauc.so on cuda:0: world 1 in-process, world 2 as two
processes sharing cuda:0 with the gloo backend (CUDA tensors), since the GPU
box has one device.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch

import coda_parity

pytestmark = pytest.mark.gpu


def _load(golden, world):
    with np.load(golden / f"coda_w{world}.npz") as z:
        return {k: z[k] for k in z.files}


def test_coda_round_world1(dev, golden):
    fx = _load(golden, 1)
    rec, _ = coda_parity.run_rank(fx, 0, 1, dev)
    coda_parity.compare(fx, 0, rec)


def test_coda_round_world1_fused_softmax_head(dev, golden):
    """Same trajectory with the softmax column folded into the surrogate kernel."""
    fx = _load(golden, 1)
    rec, _ = coda_parity.run_rank(fx, 0, 1, dev, head="logits")
    coda_parity.compare(fx, 0, rec)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, golden_dir, errq):
    import torch.distributed as dist
    from pathlib import Path

    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        fx = _load(Path(golden_dir), world)
        rec, _ = coda_parity.run_rank(fx, rank, world, torch.device("cuda", 0))
        coda_parity.compare(fx, rank, rec)
        dist.destroy_process_group()
        errq.put((rank, None))
    except BaseException as e:  # report to the parent
        import traceback

        errq.put((rank, traceback.format_exc()))
        raise SystemExit(1) from e


@pytest.mark.timeout(240)
def test_coda_round_world2_gloo_on_device(dev, golden):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(golden), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(200)
    errs = []
    while not q.empty():
        errs.append(q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    bad = [e for _, e in errs if e]
    assert not bad, "\n".join(bad)
    assert len(errs) == 2 and all(p.exitcode == 0 for p in procs)
