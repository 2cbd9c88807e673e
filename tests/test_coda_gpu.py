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


def _load(golden, world, suffix=""):
    with np.load(golden / f"coda_w{world}{suffix}.npz") as z:
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


def test_checkpoint_resume_bitwise(dev, golden, tmp_path):
    """Stop after step 5 (mid stage 2), save, restore into a fresh CoDA, finish: identical to one run."""
    import json as _json

    import tinynet
    from distributedauc_amd.coda import CoDA

    fx = _load(golden, 1)
    cfg = _json.loads(str(fx["config"]))
    xs, ys = fx["r0_x"], fx["r0_y"]

    def make():
        net = tinynet.TinyNet()
        net.load_state_dict({k[5:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("init_")})
        return CoDA(net.to(dev), lr=cfg["lr"], gamma=cfg["gamma"], T0=cfg["T0"], I=cfg["I"],
                    split_index=cfg["split_index"], device=dev)

    def stream(start=0):
        for k in range(start, len(xs)):
            yield torch.from_numpy(xs[k]).to(dev), torch.from_numpy(ys[k]).to(dev)

    full = make()
    full.run(stream(), num_stages=cfg["numStages"], total_iter=cfg["total_iter"])

    class Stop(Exception):
        pass

    used = {"n": 0}

    def counting(it):
        for b in it:
            used["n"] += 1
            yield b

    part = make()
    ck = str(tmp_path / "coda.pt")

    def stop_at(c):
        if c.t_total == 5:
            c.save(ck)
            raise Stop

    try:
        part.run(counting(stream()), num_stages=cfg["numStages"], total_iter=cfg["total_iter"], on_step=stop_at)
    except Stop:
        pass
    resumed = make()
    resumed.load(ck)
    assert resumed.t_total == 5 and resumed.stage == 2
    resumed.run(stream(used["n"]), num_stages=cfg["numStages"], total_iter=cfg["total_iter"])
    assert torch.equal(resumed.state.flat, full.state.flat)
    assert torch.equal(resumed.state.avg, full.state.avg)
    assert torch.equal(resumed.state.gcounts, full.state.gcounts)
    assert resumed.t_total == full.t_total


def test_coda_graph_replay_matches_eager_and_reference(dev, golden):
    """CoDA.use_graph(): every step body replayed from one HIP graph (re-captured when the stage
    changes lr) gives the eager run's trajectory bit for bit — parameters, a/b/alpha, counts,
    p_hat, losses, BN buffers — and so the reference's, over 2 stages with averaging rounds."""
    fx = _load(golden, 1)
    eager, _ = coda_parity.run_rank(fx, 0, 1, dev)
    graphed, coda = coda_parity.run_rank(fx, 0, 1, dev, graph=True)
    assert coda._graph is not None
    for k in eager:
        assert np.array_equal(eager[k], graphed[k]), k
    coda_parity.compare(fx, 0, graphed)


def test_coda_graph_eager_update_matches_eager_and_reference(dev, golden):
    """use_graph(eager_update=True) (the bench's headline mode): label map -> forward -> surrogate
    -> backward replayed from one graph, the update launched eagerly from the replay's static
    gradient buffers. Same trajectory as eager, bit for bit, over 2 stages (lr not baked in: ONE
    capture), and the reference's; switching back to eager steps afterwards stays exact."""
    fx = _load(golden, 1)
    eager, _ = coda_parity.run_rank(fx, 0, 1, dev)
    graphed, coda = coda_parity.run_rank(fx, 0, 1, dev, graph=True, eager_update=True)
    assert coda._graph is not None and coda.graph_captures == 1
    for k in eager:
        assert np.array_equal(eager[k], graphed[k]), k
    coda_parity.compare(fx, 0, graphed)
    # leaving graph mode: the static gradient buffers are dropped, eager backward starts from None
    assert all(p.grad is not None for p in coda.model.parameters())
    coda.use_graph(False)
    assert all(p.grad is None for p in coda.model.parameters())


def test_step_body_hip_graph_bitwise(dev, golden):
    """CoDA.step_body (label map, forward, surrogate, backward, pd_update, zero_grad) captured in a
    HIP graph and replayed 3 times from a saved state gives the same parameters, running average,
    class counts and BN buffers, bit for bit, as 3 eager calls from that state (no host sync
    inside the step; scripts/probe_graph.py measures the ResNet-50 step the same way)."""
    import json as _json

    import tinynet
    from distributedauc_amd.coda import CoDA

    fx = _load(golden, 1)
    cfg = _json.loads(str(fx["config"]))
    net = tinynet.TinyNet()
    net.load_state_dict({k[5:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("init_")})
    coda = CoDA(net.to(dev), lr=cfg["lr"], gamma=cfg["gamma"], T0=cfg["T0"], I=cfg["I"],
                split_index=cfg["split_index"], device=dev)
    batches = ((torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)) for x, y in zip(fx["r0_x"], fx["r0_y"]))
    coda.average_all()
    coda.begin_stage(1, batches)
    x, y = next(batches)
    st = coda.state
    state = [st.flat, st.avg, st.lcounts, st.gcounts, *net.buffers()]
    snap = [t.clone() for t in state]

    def restore():
        for t, s in zip(state, snap):
            t.copy_(s)

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            coda.step_body(x, y)
    torch.cuda.current_stream(dev).wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        coda.step_body(x, y)
    torch.cuda.synchronize(dev)

    restore()
    for _ in range(3):
        coda.step_body(x, y)
    eager = [t.clone() for t in state]
    restore()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize(dev)
    for e, g in zip(eager, state):
        assert torch.equal(e, g)
    assert not torch.equal(eager[0], snap[0])  # the steps did move the parameters


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, golden_dir, errq, suffix=""):
    import torch.distributed as dist
    from pathlib import Path

    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        fx = _load(Path(golden_dir), world, suffix)
        rec, _ = coda_parity.run_rank(fx, rank, world, torch.device("cuda", 0))
        coda_parity.compare(fx, rank, rec)
        dist.destroy_process_group()
        errq.put((rank, None))
    except BaseException as e:  # report to the parent
        import traceback

        errq.put((rank, traceback.format_exc()))
        raise SystemExit(1) from e


@pytest.mark.parametrize("world,suffix", [(2, ""), (8, "_I8_s4")])
@pytest.mark.timeout(300)
def test_coda_round_gloo_on_device(dev, golden, world, suffix):
    """world ranks as gloo processes sharing cuda:0, the HIP kernels doing every step, vs the
    reference's trajectory at that world size (8 ranks, I = 8: BASELINE configs[2]'s shape)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(golden), q, suffix)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(260)
    errs = []
    while not q.empty():
        errs.append(q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    bad = [e for _, e in errs if e]
    assert not bad, "\n".join(bad)
    assert len(errs) == world and all(p.exitcode == 0 for p in procs)
