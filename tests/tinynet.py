"""Tiny deterministic backbone + data stream for the CoDA-round parity fixture.

A full ResNet round cannot match a CPU run to 1e-5 (backbone conv kernels
differ), so round parity is proven on this small fp32 network that still has
every ingredient the reference path touches: Linear weights and biases,
BatchNorm affine parameters AND running buffers (which the reference does not
average, main.py:35), and the softmax head whose column 1 is the score
(resnet.py:159, 218).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

D_IN = 6
HIDDEN = 8
BATCH = 8
NUM_CLASSES = 10
SPLIT_INDEX = 7  # classes 8, 9 are positive -> ~20 % positives


class TinyNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(D_IN, HIDDEN)
        self.bn = nn.BatchNorm1d(HIDDEN)
        self.fc2 = nn.Linear(HIDDEN, 2)
        self.softmax = nn.Softmax(dim=1)

    def forward(self, x):
        return self.softmax(self.fc2(torch.relu(self.bn(self.fc1(x)))))


def make_batches(rank: int, count: int, seed: int = 123):
    """Per-rank deterministic batches: x ~ N(0,1) [BATCH, D_IN] fp32, class labels int64."""
    rng = np.random.default_rng(seed * 1000 + rank)
    xs = rng.standard_normal((count, BATCH, D_IN)).astype(np.float32)
    ys = rng.integers(0, NUM_CLASSES, size=(count, BATCH)).astype(np.int64)
    return xs, ys


def initial_state(seed: int = 1234) -> dict:
    torch.manual_seed(seed)
    net = TinyNet()
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


# the configuration the fixture was generated with
CONFIG = dict(T0=3, numStages=3, I=2, lr=0.1, gamma=10.0, total_iter=10_000, split_index=SPLIT_INDEX)
