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
