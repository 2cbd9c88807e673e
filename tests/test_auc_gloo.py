"""The sharded exact-AUC orchestration on CPU (gloo, world 2 and 3): every rank compacts the
positives of its slice of the labels into a slot, one all-gather of the slots, every rank counts
the next rank's slice of the scores against the gathered table, one all-gather of the 8-word part
records, counts summed on the host; ranks whose labels, positive scores or lengths differ raise
together; a slot that overflows (an unshuffled test set) and a table the index cannot hold take
the sorted path on every rank. Below
ExactAUC.SHARD_MIN scores every rank evaluates the whole vector instead (same integers, no
collective); both modes run here. The kernels are served by the oracle (tests/cpu_kernels.py);
the GPU form runs in bench.py --gpus 2 (tests/test_bench_gpu.py)."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

import cpu_kernels
from test_coda_gloo import _free_port


def _worker(rank, world, port, q, shard_min):
    import traceback

    import torch.distributed as dist

    try:
        torch.set_num_threads(1)
        cpu_kernels.install_in_process()
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributedauc_amd.auc import ExactAUC
        from oracle import coracle

        rng = np.random.default_rng(5)
        rng2 = np.random.default_rng(9)
        n = 20_011
        s = (np.floor(rng.random(n) * 997) / 997).astype(np.float32)
        y = np.where(rng.random(n) < 0.03, 1, -1).astype(np.int8)
        ev = ExactAUC(world=world, rank=rank, method="sort", shard_min=shard_min)
        c = ev.counts(torch.from_numpy(y), torch.from_numpy(s), device="cpu")
        assert ev.last_mode == ("sharded" if n >= shard_min else "replicated"), ev.last_mode
        e = coracle.auc_counts(y.astype(np.int64), s)
        assert (c["wins"], c["ties"], c["P"], c["N"]) == (e["wins"], e["ties"], e["P"], e["N"]), (c, e)
        # labels beyond {-1, 1}: sklearn's roc_curve(pos_label=1) takes every label other than 1 as a
        # negative ("multiclass" y_true is accepted when pos_label is given), so the counts, and the
        # AUC, are sklearn's; "other" reports how many labels lay outside {-1, 1}
        ym = y.astype(np.int32)
        ym[::7] = 0
        ym[3::11] = 2
        cm = ev.counts(torch.from_numpy(ym), torch.from_numpy(s), device="cpu")
        em = coracle.auc_counts(ym.astype(np.int64), s)
        assert (cm["wins"], cm["ties"], cm["P"], cm["N"]) == (em["wins"], em["ties"], em["P"], em["N"]), (cm, em)
        assert cm["other"] == int(((ym != 1) & (ym != -1)).sum())
        from oracle import reference_cpu as R

        assert abs(ExactAUC.from_counts(cm) - R.auc_sklearn(ym, s)) <= 1e-12
        # a non-finite negative in one rank's slice is seen by every rank after the reduce
        s2 = s.copy()
        s2[np.flatnonzero(y == -1)[-3]] = np.nan
        try:
            ev.counts(torch.from_numpy(y), torch.from_numpy(s2), device="cpu")
            raised = False
        except ValueError:
            raised = True
        assert raised
        if ev.last_mode == "sharded":
            # ranks holding different labels: every rank checks its own labels over the
            # next rank's slice against the slot that rank compacted from it -- all raise together.
            # (Labels a rank holds but never reads -- outside its own and the next slice -- cannot
            # change the result and are not checked.) Indices 10000-13000: rank 1's own slice at
            # world 2 and 3, queried by rank 0.
            y3 = y.copy()
            if rank == 1:
                neg = np.flatnonzero(y == -1)
                y3[neg[(neg > 10_000) & (neg < 13_000)][:4]] = 1
            with pytest.raises(RuntimeError, match="disagree"):
                ev.counts(torch.from_numpy(y3), torch.from_numpy(s), device="cpu")
            # ranks called with different lengths: equal slot sizes, so the gather completes and
            # every rank raises
            m = n if rank == 0 else n - 300
            with pytest.raises(RuntimeError, match="different lengths"):
                ev.counts(torch.from_numpy(y[:m].copy()), torch.from_numpy(s[:m].copy()), device="cpu")
            # the group is still usable: the same exact counts
            c2 = ev.counts(torch.from_numpy(y), torch.from_numpy(s), device="cpu")
            assert c2 == c, (c2, c)
            # an unshuffled test set: every positive in rank 0's slice overflows its slot -- the
            # sorted path on every rank, same integers
            y5 = np.where(np.arange(n) < 8000, 1, -1).astype(np.int8)  # P <= n / 2 + 1: the index could hold it
            c5 = ev.counts(torch.from_numpy(y5), torch.from_numpy(s), device="cpu")
            e5 = coracle.auc_counts(y5.astype(np.int64), s)
            assert (c5["wins"], c5["ties"], c5["P"]) == (e5["wins"], e5["ties"], e5["P"])
            # a table the index cannot hold (positives > n / 2 + 1 here): the sorted path, same integers
            y4 = np.where(rng2.random(n) < 0.7, 1, -1).astype(np.int8)
            c4 = ev.counts(torch.from_numpy(y4), torch.from_numpy(s), device="cpu")
            e4 = coracle.auc_counts(y4.astype(np.int64), s)
            assert (c4["wins"], c4["ties"], c4["P"]) == (e4["wins"], e4["ties"], e4["P"])
        dist.destroy_process_group()
        q.put((rank, None))
    except BaseException:
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("shard_min", [0, 1 << 25])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.timeout(300)
def test_sharded_sort_auc_gloo(world, shard_min):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, shard_min)) for r in range(world)]
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


def _pairs_worker(rank, world, port, q):
    import traceback

    import torch.distributed as dist

    try:
        torch.set_num_threads(1)
        cpu_kernels.install_in_process()
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributedauc_amd.auc import ExactAUC
        from oracle import coracle

        rng = np.random.default_rng(11)
        n = 3_001
        s = (np.floor(rng.random(n) * 211) / 211).astype(np.float32)
        y = np.where(rng.random(n) < 0.05, 1, -1).astype(np.int8)
        ev = ExactAUC(world=world, rank=rank, method="pairs")
        c = ev.counts(torch.from_numpy(y), torch.from_numpy(s), device="cpu")
        e = coracle.auc_counts(y.astype(np.int64), s)
        assert (c["wins"], c["ties"], c["P"], c["N"]) == (e["wins"], e["ties"], e["P"], e["N"]), (c, e)
        # a non-finite score: every rank raises after the gather (none is left in the collective)
        s2 = s.copy()
        s2[7] = np.inf
        with pytest.raises(ValueError, match="NaN or infinity"):
            ev.counts(torch.from_numpy(y), torch.from_numpy(s2), device="cpu")
        # ranks holding different vectors: every rank raises
        y3 = y.copy()
        if rank == 1:
            y3[np.flatnonzero(y == -1)[:4]] = 1
        with pytest.raises(RuntimeError, match="disagree"):
            ev.counts(torch.from_numpy(y3), torch.from_numpy(s), device="cpu")
        # and the group is still usable afterwards: the same exact counts
        c2 = ev.counts(torch.from_numpy(y), torch.from_numpy(s), device="cpu")
        assert c2 == c, (c2, c)
        dist.destroy_process_group()
        q.put((rank, None))
    except BaseException:
        q.put((rank, traceback.format_exc()))


@pytest.mark.timeout(300)
def test_sharded_pairs_auc_gloo():
    """The pair-count method over world 2: positive blocks sharded, one all-gather of the
    per-rank (W, T, P, N, non-finite, other) records; inconsistent or non-finite inputs raise on
    every rank together (no rank may raise while the others wait in the collective)."""
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_pairs_worker, args=(r, world, port, q)) for r in range(world)]
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
