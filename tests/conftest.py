import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
# the shipped MI355X MIOpen find/perf db (ResNet-50 b256 convolutions), set before any GPU test
# runs a convolution, as bench.py and main.train do
from distributedauc_amd import use_tuned_miopen_db  # noqa: E402

use_tuned_miopen_db()

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdauc.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running (large sizes)")


@pytest.fixture(scope="session")
def dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def golden():
    return GOLDEN
