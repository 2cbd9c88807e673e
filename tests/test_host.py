"""Host-side surface: CLI flags, partitioner (reference + stratified), data labels, backbone, layout."""
from __future__ import annotations

import hashlib
import json

import numpy as np
import pytest
import torch

from distributedauc_amd import backbone, data_partitioner, loader, parameters
from distributedauc_amd.flat import ALIGN, FlatState, _dense_layout, _same_order


def test_reference_flags_and_defaults():
    """parameters.py:5-23 of the reference: every flag, same default."""
    p = parameters.parse([])
    ref = dict(T0=5000, numStages=10000, local_batchsize=32, lr=0.1, gamma=2000, test_freq=800, test_batchsize=32,
               test_batches=100, save_freq=10000, I=2, split_index=4, numGPU=1, total_iter=2000, neg_keep_ratio=1,
               local_rank=0, master_addr=None, test_ratio=0.0001)
    for k, v in ref.items():
        assert getattr(p, k) == v, k
    q = parameters.parse("--T0=5000 --gamma=2000 --lr=0.1 --I=64 --local_batchsize=32 --neg_keep_ratio=0.4 "
                         "--total_iter=40000 --split_index=499 --test_ratio=0.01".split())  # node0.sh:4-5
    assert (q.I, q.neg_keep_ratio, q.split_index, q.test_ratio) == (64, 0.4, 499, 0.01)


class _Len:
    def __len__(self):
        return data_partitioner.IMAGENET_LEN


@pytest.mark.parametrize("keep,size", [(0.4, 1), (0.4, 2), (0.4, 8), (0.4, 16), (1.0, 4), (1.0, 16)])
def test_reference_partitions_bit_exact(golden, keep, size):
    ref = json.loads((golden / "partitions.json").read_text())[f"keep{keep}_size{size}"]
    part = data_partitioner.DataPartitioner(_Len(), data_partitioner.partition_sizes(size, 0.01), seed=123,
                                            neg_keep_ratio=keep, mode="reference")
    assert len(part.partitions) == len(ref)
    for p, r in zip(part.partitions, ref):
        assert len(p) == r["len"] and [int(v) for v in p[:5]] == r["head"]
        assert hashlib.sha256(np.asarray(p, np.int64).tobytes()).hexdigest() == r["sha256"]


def test_stratified_partitions_preserve_imbalance():
    labels = loader.imagenet_like_labels(200_000, 1000, 499, pos_ratio=0.1, seed=3)
    sizes = data_partitioner.partition_sizes(8, 0.01)
    part = data_partitioner.DataPartitioner(labels, sizes, seed=123, neg_keep_ratio=0.4, mode="stratified",
                                            labels=labels, split_index=499)
    allidx = np.concatenate([np.asarray(p) for p in part.partitions])
    assert len(np.unique(allidx)) == len(allidx)  # disjoint
    fracs = [np.mean(labels[np.asarray(p)] > 499) for p in part.partitions[1:]]
    n_pos = np.sum(labels > 499)
    n_neg = int((len(labels) - n_pos) * 0.4)
    expect = n_pos / (n_pos + n_neg)
    assert max(abs(f - expect) for f in fracs) < 2e-4  # every rank trains at the global rate
    assert abs(len(part.use(0)) - 0.01 * (n_pos + n_neg)) < 3


def test_stratified_needs_labels():
    with pytest.raises(ValueError):
        data_partitioner.DataPartitioner(_Len(), [0.5, 0.5], mode="stratified")


def test_imagenet_like_labels_match_reference_ranges():
    lab = loader.imagenet_like_labels()
    assert lab.shape == (1281167,)
    assert lab[: 642289].max() <= 499 and lab[642290:].min() > 499
    assert lab.min() == 0 and lab.max() == 999


@pytest.mark.parametrize("arch,n,t", [("resnet18", 11177538, 62), ("resnet50", 23512130, 161)])
def test_backbone_parameter_counts(arch, n, t):
    net = backbone.build_backbone(arch)
    assert sum(p.numel() for p in net.parameters()) == n  # SURVEY §2 [probed] counts
    assert len(list(net.parameters())) == t
    out = net.eval()(torch.randn(2, 3, 64, 64))
    assert out.shape == (2, 2) and torch.allclose(out.sum(1), torch.ones(2))  # softmax head


def test_dense_layout_and_flat_requires_gpu():
    assert _dense_layout(torch.zeros(3, 4, 5, 6).contiguous(memory_format=torch.channels_last))
    assert not _dense_layout(torch.zeros(4, 6)[:, ::2])
    with pytest.raises(RuntimeError, match="GPU memory"):
        FlatState(torch.nn.Linear(3, 2))
    assert ALIGN * 4 == 256


def test_gradient_memory_order_check():
    """FlatState.grad_segments copies a gradient only when its memory order differs from the
    parameter's: a 1x1 conv weight's contiguous gradient is the channels-last parameter's order."""
    p1 = torch.empty_strided((8, 4, 1, 1), (4, 1, 4, 4))  # what model.to(channels_last) leaves
    assert p1.stride() != torch.zeros(8, 4, 1, 1).stride()
    assert _same_order(torch.zeros(8, 4, 1, 1), p1)
    p3 = torch.zeros(8, 4, 3, 3).contiguous(memory_format=torch.channels_last)
    assert not _same_order(torch.zeros(8, 4, 3, 3), p3)
    assert _same_order(torch.zeros(8, 4, 3, 3).contiguous(memory_format=torch.channels_last), p3)
    assert not _same_order(torch.zeros(8, 8)[:, ::2], torch.zeros(8, 4))
    assert not _same_order(torch.zeros(4, 8).t(), torch.zeros(8, 4))


def test_run_label_format():
    from distributedauc_amd.main import run_label

    p = parameters.parse("--split_index 499 --neg_keep_ratio 0.4 --I 64".split())
    s = run_label(p, 16)
    assert s.startswith("_size_16_lr_0.1_T0_5000_gamma_2000_p_0.71_I_64_local_batchsize_32")
