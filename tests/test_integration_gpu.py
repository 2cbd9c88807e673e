"""The reference-side ctypes binding shown in INTEGRATION.md §2, executed verbatim against libdauc.so:
its AUC() (the one blocking call dauc_auc_eval_counts) must give the C oracle's exact counts, its
dppd_sg_param() the oracle's bit-exact update (main.py:61), and its AUC_sharded() -- through 2 gloo
ranks on cuda:0 at configs[3]'s 2^24 scores -- the oracle's counts on both ranks, with ranks that
hold different labels or lengths raising together. Reference: main.py:79-81,
232-250; sklearn _ranking.py:826-908."""
from __future__ import annotations

import os
import re
import socket
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import coracle

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _stub():
    text = (REPO / "INTEGRATION.md").read_text()
    sec = text[text.index("## 2. Bind the C ABI directly"):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    os.environ["DAUC_LIB"] = str(REPO / "distributedauc_amd" / "libdauc.so")
    ns: dict = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    return ns


def test_integration_stub_auc_and_update(dev):
    ns = _stub()
    rng = np.random.default_rng(11)
    for n, p, q in ((1000, 0.1, 0), (300_007, 0.01, 1024), (300_007, 0.9, 1024), (2_000_000, 0.002, 0)):
        s = rng.random(n, dtype=np.float32)
        if q:
            s = (np.floor(s * q) / q).astype(np.float32)
        y = np.where(rng.random(n) < p, 1, -1).astype(np.int8)
        e = coracle.auc_counts(y.astype(np.int64), s)
        got = ns["AUC"](torch.from_numpy(y), torch.from_numpy(s))
        assert got == (2 * e["wins"] + e["ties"]) / (2 * e["P"] * e["N"])
    y[5], s[5] = -1, np.nan  # a non-finite negative: only the query pass sees it
    with pytest.raises(ValueError):
        ns["AUC"](torch.from_numpy(y), torch.from_numpy(s))
    w, g, w0 = (rng.standard_normal(4099).astype(np.float32) for _ in range(3))
    tw = torch.from_numpy(w).to(dev)
    tw.grad = torch.from_numpy(g).to(dev)
    ns["dppd_sg_param"](tw, torch.from_numpy(w0).to(dev), 0.1, 2000.0)
    torch.cuda.synchronize()
    assert np.array_equal(tw.cpu().numpy(), coracle.pd_update(w, g, w0, 0.1, 2000.0))


def _area(e):
    return (2 * e["wins"] + e["ties"]) / (2 * e["P"] * e["N"])


def _sharded_worker(rank, world, port, q):
    import traceback

    import torch.distributed as dist

    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributedauc_amd.loader import synthetic_scores

        ns = _stub()
        auc = ns["AUC_sharded"]
        ts, ty = synthetic_scores(1 << 24, 0.01, dev)
        s, y = ts.cpu().numpy(), ty.cpu().numpy().astype(np.int64)
        e = coracle.auc_counts(y, s)
        assert auc(ty, ts) == _area(e)
        assert auc(ty, ts) == ns["AUC"](ty, ts)
        # labels outside {-1, 1} are negatives (sklearn's pos_label=1)
        ym = ty.to(torch.int32)
        ym[::5] = torch.where(ym[::5] == 1, 1, 0)
        em = coracle.auc_counts(ym.cpu().numpy().astype(np.int64), s)
        assert auc(ym, ts) == _area(em)
        # ranks whose labels differ in a slice another rank reads: both raise after the collectives
        y3 = ty.clone()
        if rank == 1:
            y3[(1 << 23) + 777:(1 << 23) + 777 + 64] = 1
        with pytest.raises(RuntimeError, match="disagree"):
            auc(y3, ts)
        # different lengths: equal slot sizes, the gathers complete, both raise
        m = (1 << 24) - (0 if rank == 0 else 4096)
        with pytest.raises(RuntimeError, match="different lengths"):
            auc(ty[:m], ts[:m])
        # a non-finite negative in one slice: both raise
        s4 = ts.clone()
        s4[int(torch.nonzero(ty == -1)[-5])] = float("nan")
        with pytest.raises(ValueError):
            auc(ty, s4)
        # an unshuffled test set (every positive in rank 0's slice overflows its slot): verdict 2,
        # the blocking sorted path on both ranks, the oracle's integers
        y5 = torch.where(torch.arange(1 << 24, device=dev) < 200_000, 1, -1).to(torch.int8)
        e5 = coracle.auc_counts(y5.cpu().numpy().astype(np.int64), s)
        assert auc(y5, ts) == _area(e5)
        # tie-heavy scores (bf16-rounded): verdict 2, then dauc_auc_eval_query_part_sorted over the
        # gathered slots on both ranks (the distinct-key index), the oracle's integers
        tb = ts.bfloat16().float()
        eb = coracle.auc_counts(y, tb.cpu().numpy())
        assert auc(ty, tb) == _area(eb)
        assert auc(ty, ts) == _area(e)  # the group is still usable
        dist.destroy_process_group()
        q.put((rank, None))
    except BaseException:
        q.put((rank, traceback.format_exc()))


@pytest.mark.timeout(400)
def test_integration_stub_sharded_two_gloo_ranks_2e24():
    """INTEGRATION.md §2's AUC_sharded, verbatim, as 2 processes on cuda:0 over gloo at 2^24 scores
    and 1 % positives (configs[3]): the oracle's counts; multi-valued labels as sklearn; differing
    labels, lengths and a non-finite score raise on both ranks; the verdict-2 paths (tie-heavy
    scores through the sorted two-step fallback, an unshuffled set through the whole-vector one)."""
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(360)
    res = []
    while not q.empty():
        res.append(q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = [e for _, e in res if e]
    assert not errs, "\n".join(errs)
    assert sorted(r for r, _ in res) == list(range(world))
