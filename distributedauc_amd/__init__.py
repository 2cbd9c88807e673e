"""distributedauc_amd — MI355X-native hot path of CoDA distributed AUC maximization.

A drop-in for the data-parallel AUC path of ZhishuaiGuo/DistributedAUC
(imagenet/main.py): the min-max square-loss surrogate, the proximal
primal-dual update over the flattened model, CoDA periodic averaging over
RCCL, and exact AUC evaluation. The AUC-specific work runs in hand-written
gfx950 HIP kernels behind the C ABI of include/dauc.h (libdauc.so); the ResNet
backbone stays on PyTorch-ROCm.
"""
from . import _lib

__version__ = "1.0.0"

__all__ = ["_lib", "ops", "auc", "coda", "flat", "surrogate", "backbone", "main", "parameters",
           "data_partitioner", "loader"]


def __getattr__(name):  # lazy submodules: importing the package does not need a GPU
    import importlib

    if name in __all__:
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
