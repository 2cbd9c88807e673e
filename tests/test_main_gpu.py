"""The reference-compatible driver end to end on the GPU: main.train() with a tiny config.

Covers the CLI surface, the stratified partitioner, the on-device loader, the
CoDA schedule with evaluation every test_freq steps (main.py:215), the sharded
exact AUC, and the history CSV of main.py:252-261 (columns total_iteration,
time, Test<configs>).
"""
from __future__ import annotations

import math

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
@pytest.mark.parametrize("head", ["softmax", "logits"])
def test_main_train_tiny(dev, tmp_path, head):
    import pandas as pd

    from distributedauc_amd import main as M
    from distributedauc_amd.parameters import parse

    para = parse(["--arch", "resnet18", "--image_size", "32", "--dataset_size", "6000", "--num_classes", "10",
                  "--split_index", "6", "--pos_ratio", "0.3", "--T0", "4", "--numStages", "3", "--I", "2",
                  "--local_batchsize", "16", "--test_batchsize", "64", "--test_freq", "3", "--total_iter", "100",
                  "--test_ratio", "0.05", "--history_dir", str(tmp_path), "--neg_keep_ratio", "0.5"])
    para.head = head
    coda = M.train(0, 1, None, para)
    assert coda.t_total == 4 + 12  # T0 * (1 + 3) steps over stages 1 and 2
    files = list(tmp_path.glob("history*.csv"))
    assert len(files) == 1
    df = pd.read_csv(files[0], index_col=0)
    assert list(df.columns[:2]) == ["total_iteration", "time"] and df.columns[2].startswith("Test_size_1_")
    assert list(df["total_iteration"]) == [0, 3, 6, 9, 12, 15]
    assert all(0.0 <= a <= 1.0 and not math.isnan(a) for a in df.iloc[:, 2])


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _split_eval_worker(rank, world, port, errq):
    import os
    import sys
    from pathlib import Path

    import torch
    import torch.distributed as dist

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    try:
        from distributedauc_amd import main as M
        from distributedauc_amd.parameters import parse

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        checked = {"n": 0}

        class Checked(M.Evaluator):
            """Every evaluation twice: split scoring, then the reference's rank-0 scoring."""

            def __call__(self, coda):
                st = coda.state
                bufs = list(coda.model.buffers())
                flat0, bufs0 = st.flat.clone(), [b.clone() for b in bufs]
                self.split_scoring = True
                a_split = super().__call__(coda)
                s_split = self.last_scores.clone()
                assert torch.equal(st.flat, flat0), f"rank {rank}: own parameters not restored"
                assert all(torch.equal(b, c) for b, c in zip(bufs, bufs0)), f"rank {rank}: BN buffers not restored"
                self.split_scoring = False
                a_ref = super().__call__(coda)
                ref = self.last_scores
                if not torch.equal(s_split, ref):
                    bad = (s_split != ref).nonzero().flatten().tolist()
                    sizes = [lab.numel() for _, lab in self.batches]
                    raise AssertionError(f"rank {rank}: split scores differ at {len(bad)} of {ref.numel()} "
                                         f"(first {bad[:8]}, batch sizes {sizes}, shares {self._share}, "
                                         f"max diff {float((s_split - ref).abs().max())})")
                assert a_split == a_ref, (a_split, a_ref)
                self.split_scoring = True
                checked["n"] += 1
                return a_split

        M.Evaluator = Checked
        para = parse(["--arch", "resnet18", "--image_size", "32", "--dataset_size", "6000", "--num_classes", "10",
                      "--split_index", "6", "--pos_ratio", "0.3", "--T0", "4", "--numStages", "3", "--I", "3",
                      "--local_batchsize", "16", "--test_batchsize", "48", "--test_freq", "5", "--total_iter", "100",
                      "--test_ratio", "0.1", "--history_dir", "", "--neg_keep_ratio", "0.5",
                      "--deterministic_eval", "1"])
        coda = M.train(rank, world, None, para)
        assert checked["n"] >= 2, checked
        dist.barrier()
        dist.destroy_process_group()
        errq.put((rank, None))
    except BaseException as e:
        import traceback

        errq.put((rank, traceback.format_exc()))
        raise SystemExit(1) from e


@pytest.mark.timeout(400)
def test_main_split_scoring_world2(dev):
    """World 2 (gloo ranks on cuda:0) with averaging every 3 steps and an evaluation every 5, so
    the ranks hold different parameters and BN statistics when they evaluate: the test set scored
    in two shares with rank 0's broadcast model gives bit-identical scores and the same AUC as
    rank 0 scoring it all, and each rank's own model is restored afterwards."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_split_eval_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(360)
    errs = []
    while not q.empty():
        errs.append(q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    bad = [e for _, e in errs if e]
    assert not bad, "\n".join(bad)
    assert len(errs) == 2 and all(p.exitcode == 0 for p in procs)
