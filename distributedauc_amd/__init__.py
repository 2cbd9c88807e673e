"""distributedauc_amd — MI355X-native hot path of CoDA distributed AUC maximization.

A drop-in for the data-parallel AUC path of ZhishuaiGuo/DistributedAUC
(imagenet/main.py): the min-max square-loss surrogate, the proximal
primal-dual update over the flattened model, CoDA periodic averaging over
RCCL, and exact AUC evaluation. The AUC-specific work runs in hand-written
gfx950 HIP kernels behind the C ABI of include/dauc.h (libdauc.so). The ResNet
backbone runs on PyTorch-ROCm (MIOpen / CK convolutions, hipBLASLt GEMMs) with
some of its passes on the same library's HIP kernels when switched on
(backbone.py: fused BN + add + ReLU, the stem max-pool, the bf16 weight shadow
with the 3x3 and 7x7-stem weight-gradient and stem-forward MFMA kernels, the
strided / broadcast copies; CoDA turns them on under bf16 autocast and bench.py
uses them); each is parity-tested against an fp64 / torch reference of its op.
"""
import os

from . import _lib

__version__ = "1.0.0"

MIOPEN_DB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "miopen_db")


def use_tuned_miopen_db() -> str:
    """Point MIOpen at the shipped MI355X find + perf db unless the caller already chose one
    (MIOPEN_USER_DB_PATH). The db holds the ResNet-50 b256 channels-last bf16 convolutions of
    bench.py tuned by exhaustive search (torch.backends.cudnn.benchmark, scripts/gpu_miopen_tune.sh):
    27.2 vs 28.5 ms per backbone step, and ~1 s instead of ~60 s of first-step solver search.
    Call before the first convolution; returns the db path in effect."""
    return os.environ.setdefault("MIOPEN_USER_DB_PATH", MIOPEN_DB)

__all__ = ["_lib", "ops", "auc", "coda", "flat", "surrogate", "backbone", "main", "parameters",
           "data_partitioner", "loader"]


def __getattr__(name):  # lazy submodules: importing the package does not need a GPU
    import importlib

    if name in __all__:
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
