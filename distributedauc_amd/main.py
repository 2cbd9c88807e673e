"""Reference-compatible host API and training entry point (imagenet/main.py).

The functions keep the reference's names, signatures and in-place semantics:

    average_model(model, group)                                        main.py:33
    average_all(model, a, b, alpha, gpos, gneg, lpos, lneg, group)     main.py:40
    dppd_sg(model, a, b, alpha, model0, a0, b0, alpha0, lr, gamma)     main.py:56
    AUC(label, scores)                                                 main.py:79
    train(rank, size, group)                                           main.py:83

When the model was flattened by ``CoDA``/``FlatState`` and a, b, alpha are its
views, ``average_all`` and ``dppd_sg`` take the one-launch flat path. Otherwise
they walk the tensors like the reference does, still through the HIP kernels
(one launch per tensor). Launch (replaces node0..3.sh): one process per GPU,

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m distributedauc_amd.main --I 16 ...
"""
from __future__ import annotations

import os
import random
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from . import ops
from .auc import AUC as _gpu_auc
from .auc import ExactAUC
from .backbone import build_backbone
from .coda import CoDA
from .data_partitioner import DataPartitioner, partition_sizes
from .loader import DeviceLoader, SyntheticImageNet, imagenet_like_labels
from .parameters import parse


def _world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _flat_of(model, a):
    st = getattr(model, "_dauc_flat", None)
    if st is not None and a is not None and a.data_ptr() == st.a.data_ptr():
        return st
    return None


# ----------------------------------------------------------------- a6
def average_model(model, group=None):
    """main.py:33-38: every parameter <- all_reduce(SUM) / world (buffers untouched)."""
    size = _world(group)
    for param in model.parameters():
        if size > 1:
            dist.all_reduce(param.data, op=dist.ReduceOp.SUM, group=group)
            ops.scale_div(param.data, float(size))


def average_all(model, a, b, alpha, global_total_pos, global_total_neg, local_total_pos, local_total_neg,
                group=None):
    """main.py:40-54, in place. Flat models: one all-reduce + one finalise launch."""
    st = _flat_of(model, a)
    size = _world(group)
    if st is not None:
        if size > 1:
            dist.all_reduce(st.flat[: st.n_reduce], op=dist.ReduceOp.SUM, group=group)
        ops.coda_finalize(st.flat, st.n_avg, size, st.lcounts, st.gcounts)
        return
    average_model(model, group)
    for t in (a, b, alpha):
        if size > 1:
            dist.all_reduce(t.data, op=dist.ReduceOp.SUM, group=group)
            ops.scale_div(t.data, float(size))
    for t in (local_total_pos, local_total_neg):
        if size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    global_total_pos += local_total_pos
    global_total_neg += local_total_neg


# ----------------------------------------------------------------- a4
def dppd_sg(model, a, b, alpha, model0, a0, b0, alpha0, lr, gamma, mode: str = "reference"):
    """main.py:56-64 (quirks included in mode="reference"). In place on model, a, b, alpha.

    Flat models take the one-launch path when model0 is None or the FlatState's
    own anchor (the stage snapshot CoDA keeps); then a0/b0/alpha0 are the anchor's.
    """
    st = _flat_of(model, a)
    if st is not None and (model0 is None or model0 is st.anchor):
        st.update(lr, gamma, mode, running_average=False)
        return
    for name, param in model.named_parameters():
        w = param.data
        if not w.is_contiguous():
            raise ValueError(f"dppd_sg generic path needs contiguous parameters ({name})")
        ops.pd_update_dense(w, param.grad.data.contiguous(), model0[name].contiguous(), None, lr=lr, gamma=gamma)
    sc = torch.cat([a.data.reshape(1), b.data.reshape(1), alpha.data.reshape(1)]).float()
    g3 = torch.cat([a.grad.reshape(1), b.grad.reshape(1), alpha.grad.reshape(1)]).float()
    an3 = torch.cat([a0.reshape(1), b0.reshape(1), alpha0.reshape(1)]).float()
    ops.pd_update(sc, sc, None, None, 0, scalars=sc, grad3=g3, anchor3=an3, lr=lr, gamma=gamma, mode=mode)
    a.data.copy_(sc[0:1].view_as(a.data))
    b.data.copy_(sc[1:2].view_as(b.data))
    alpha.data.copy_(sc[2:3].view_as(alpha.data))


# ----------------------------------------------------------------- a8
def AUC(label, scores):  # noqa: N802 (reference name)
    """main.py:79-81 on the GPU: exact integer counts -> (2W + T) / (2PN)."""
    return _gpu_auc(label, scores)


# ----------------------------------------------------------------- driver
def _seed_everything(seed: int):
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)


def run_label(para, size: int) -> str:
    """main.py:86-90: the run label used in the history file name."""
    p = CoDA.p_prior(para.split_index, para.neg_keep_ratio, para.num_classes)
    return (f"_size_{size}_lr_{para.lr}_T0_{para.T0}_gamma_{para.gamma}_p_{p:.2f}_I_{para.I}"
            f"_local_batchsize_{para.local_batchsize}_ImageNet_{para.arch}_{para.image_size}")


class Evaluator:
    """main.py:215-270: the test-set AUC of rank 0's model, written to the history CSV.

    The reference scores the whole test partition on rank 0 (main.py:232) while the other ranks
    wait. Here (``split=True``, the default over ranks) every rank scores a contiguous share of the
    test batches with rank 0's model: rank 0's parameters and BatchNorm running statistics are
    broadcast into every rank's model for the evaluation (ranks hold different parameters between
    averaging rounds, and BN buffers are never averaged, main.py:35) and each rank's own state is
    restored afterwards. The shares are all-gathered, so every rank holds rank 0's scores in the
    test-set order, and the exact count is sharded (ExactAUC). With ``deterministic=True``
    (``--deterministic_eval 1``) the scores and the AUC are bit-identical to rank-0 scoring
    (tests/test_main_gpu.py); without it they differ from it only as much as two rank-0 scorings
    do (MIOpen's default solvers vary in low bits from call to call). ``split=False`` is the
    reference's rank-0 scoring."""

    def __init__(self, test_batches, n_test: int, split_index: int, device, group, world: int, rank: int,
                 history_path: str | None = None, split: bool = True, deterministic: bool = False,
                 collective: bool | None = None):
        self.batches = test_batches
        self.n = n_test
        self.split = split_index
        # collective (default world > 1): True at world 1 rehearses the split path's broadcast and
        # all-gather on a one-rank process group
        self.collective = world > 1 if collective is None else bool(collective)
        self.split_scoring = bool(split) and self.collective
        self.deterministic = bool(deterministic)
        self.device = device
        self.world, self.rank = world, rank
        self.auc = ExactAUC(group, world, rank, collective=self.collective)
        self.group = group
        self.history_path = history_path
        self.rows: list[tuple[int, float, float]] = []
        self.train_seconds = 0.0
        self.last_eval_seconds = 0.0
        self._mark = time.perf_counter()
        sizes = [lab.numel() for _, lab in test_batches]
        nb = len(sizes)
        self._share = [(r * nb // world, (r + 1) * nb // world) for r in range(world)]
        self._counts = [sum(sizes[lo:hi]) for lo, hi in self._share]
        self._labels = None

    def _test_labels(self) -> torch.Tensor:
        if self._labels is None:
            self._labels = torch.cat([torch.where(lab > self.split, 1, -1).to(torch.int8) for _, lab in self.batches])
        return self._labels

    def _score(self, coda: CoDA, lo: int, hi: int, out: torch.Tensor) -> None:
        from .conv1x1 import fixed_engine

        coda.model.eval()
        # no per-rank timed 1x1 engine choice. MIOpen's default forward solvers are not repeatable
        # bit for bit (ResNet-18 layer2.0.conv2 at 32x32, batch 48, changes low bits from call to
        # call: scripts/probe_eval_determinism.py, profiles/r03/determinism/), so rank 0 scoring the
        # same test set twice differs in low bits as much as split scoring does; `deterministic`
        # selects repeatable solvers, making split and rank-0 scoring bit-identical (the GPU test),
        # at a large cost for 224^2 bf16 (ResNet-50, 8192 images: 61 s vs 0.48 s)
        det, bench = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
        if self.deterministic:
            torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
        try:
            with torch.no_grad(), fixed_engine("gemm"):
                k = 0
                for x, lab in self.batches[lo:hi]:
                    out[k:k + lab.numel()] = coda.scores(x)
                    k += lab.numel()
        finally:
            torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det, bench
        coda.model.train()

    def _scores_split(self, coda: CoDA) -> torch.Tensor:
        """Every rank scores its share of the batches with rank 0's model; all-gather."""
        st = coda.state
        bufs = [b for b in coda.model.buffers() if b.dtype == torch.float32]
        saved = st.flat[: st.n_params].clone(), [b.clone() for b in bufs]
        packed = torch.cat([b.reshape(-1) for b in bufs]) if bufs else None
        dist.broadcast(st.flat[: st.n_params], 0, group=self.group)  # rank 0's parameters
        if packed is not None:
            dist.broadcast(packed, 0, group=self.group)              # rank 0's BN running statistics
            off = 0
            for b in bufs:
                b.copy_(packed[off:off + b.numel()].view_as(b))
                off += b.numel()
        seg = max(self._counts)
        mine = torch.zeros(seg, dtype=torch.float32, device=self.device)
        lo, hi = self._share[self.rank]
        self._score(coda, lo, hi, mine)
        gathered = torch.empty(seg * self.world, dtype=torch.float32, device=self.device)
        dist.all_gather_into_tensor(gathered, mine, group=self.group)
        with torch.no_grad():  # this rank's own model back
            st.flat[: st.n_params].copy_(saved[0])
            for b, s in zip(bufs, saved[1]):
                b.copy_(s)
        parts = gathered.view(self.world, seg)
        return torch.cat([parts[r, : self._counts[r]] for r in range(self.world)])

    def __call__(self, coda: CoDA):
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        self.train_seconds += t0 - self._mark
        labels = self._test_labels()
        if self.split_scoring:
            scores = self._scores_split(coda)
        else:
            scores = torch.empty(self.n, dtype=torch.float32, device=self.device)
            if self.rank == 0:
                self._score(coda, 0, len(self.batches), scores)
            if self.collective:
                dist.broadcast(scores, 0, group=self.group)
        auc = self.auc(labels, scores)
        if self.rank == 0:
            p_hat = float(coda.state.p_hat.item())
            print(time.strftime("%Y-%m-%d %H:%M:%S"), f"Stage: {coda.stage}; Iter: {coda.t_total}; "
                  f"lr: {coda.lr:.3f} ; p_hat: {p_hat}; auc: {auc:.4f}", flush=True)
            self.rows.append((coda.t_total, self.train_seconds, auc))
            if self.history_path:
                import pandas as pd

                os.makedirs(os.path.dirname(self.history_path) or ".", exist_ok=True)
                it, tm, au = zip(*self.rows)
                col = "Test" + os.path.basename(self.history_path)[len("history"):-len(".csv")]
                pd.DataFrame({"total_iteration": it, "time": tm, col: au}).to_csv(self.history_path)
        torch.cuda.synchronize(self.device)
        self._mark = time.perf_counter()
        self.last_eval_seconds = self._mark - t0
        self.last_scores = scores
        return auc


def train(rank: int, size: int, group=None, para=None):
    """main.py:83-339 with synthetic on-device data; returns the CoDA object."""
    para = para or parse([])
    from . import use_tuned_miopen_db

    use_tuned_miopen_db()  # before the first convolution
    device = torch.device("cuda", para.local_rank)
    torch.cuda.set_device(device)
    _seed_everything(para.seed)
    label = run_label(para, size)
    if rank == 0:
        print("configs: " + label, flush=True)
    labels = imagenet_like_labels(para.dataset_size, para.num_classes, para.split_index, para.pos_ratio,
                                  seed=para.seed)
    dataset = SyntheticImageNet(labels, para.image_size, para.split_index)
    partition = DataPartitioner(dataset, partition_sizes(size, para.test_ratio), seed=123,
                                neg_keep_ratio=para.neg_keep_ratio, mode=para.partition, labels=labels,
                                split_index=para.split_index)
    test_part = partition.use(0)
    train_part = partition.use(rank + 1)
    train_loader = DeviceLoader(dataset, train_part.index, para.local_batchsize, device, seed=para.seed + rank,
                                channels_last=para.channels_last)
    head = getattr(para, "head", "softmax")
    net = build_backbone(para.arch, num_classes=2, head=head).to(device)
    if para.channels_last:
        net = net.to(memory_format=torch.channels_last)
        net.set_fused_bn(para.fused_bn).set_gemm_conv1x1(para.gemm_conv1x1)
    coda = CoDA(net, lr=para.lr, gamma=para.gamma, T0=para.T0, I=para.I, split_index=para.split_index,
                mode=para.mode, world=size, rank=rank, group=group,
                autocast_dtype=torch.bfloat16 if para.bf16 else None, device=device, head=head)
    evaluate = None
    if len(test_part) > 0:
        test_loader = DeviceLoader(dataset, test_part.index, para.test_batchsize, device, seed=para.seed + 999,
                                   shuffle=False, channels_last=para.channels_last)
        n_test = len(test_part)
        it = iter(test_loader)
        test_batches = [next(it) for _ in range((n_test + para.test_batchsize - 1) // para.test_batchsize)]
        hist = os.path.join(para.history_dir, "history" + label + ".csv") if para.history_dir else None
        evaluate = Evaluator(test_batches, n_test, para.split_index, device, group, size, rank, hist,
                             split=getattr(para, "split_eval", 1) != 0,
                             deterministic=getattr(para, "deterministic_eval", 0) != 0)
    coda.run(iter(train_loader), num_stages=para.numStages, total_iter=para.total_iter,
             test_freq=para.test_freq, evaluate=evaluate)
    return coda


def main(argv=None):
    para = parse(argv)
    if para.master_addr:
        os.environ["MASTER_ADDR"] = para.master_addr  # main.py:344
    if "LOCAL_RANK" in os.environ:
        para.local_rank = int(os.environ["LOCAL_RANK"])
    if "WORLD_SIZE" in os.environ:
        dist.init_process_group(para.backend or "nccl", device_id=torch.device("cuda", para.local_rank))
        size, rank = dist.get_world_size(), dist.get_rank()
    else:
        size, rank = 1, 0
    print(f"initialized, rank: {rank} size: {size}", flush=True)
    train(rank, size, None, para)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1:])
