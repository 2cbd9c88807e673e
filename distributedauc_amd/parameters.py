"""Command-line flags: the reference's surface (parameters.py:4-23) plus build extras.

Every reference flag keeps its name, type and default. Unlike the reference,
parsing is not done at import time (parameters.py:25 parses sys.argv on import);
``para`` holds the defaults and ``parse()`` parses a command line.
"""
from __future__ import annotations

import argparse


def get_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="CoDA distributed AUC maximization on MI355X")
    # ---- reference flags (parameters.py:5-23), same defaults
    p.add_argument("--T0", type=int, default=5000)
    p.add_argument("--numStages", type=int, default=10000)
    p.add_argument("--local_batchsize", type=int, default=32)
    p.add_argument("--lr", type=float, default=0.1)  # initial learning rate
    p.add_argument("--gamma", type=float, default=2000)
    p.add_argument("--test_freq", type=int, default=800)
    p.add_argument("--test_batchsize", type=int, default=32)
    p.add_argument("--test_batches", type=int, default=100)  # parsed, never read (as in the reference)
    p.add_argument("--save_freq", type=int, default=10000)   # parsed, never read (as in the reference)
    p.add_argument("--I", type=int, default=2)
    p.add_argument("--split_index", type=int, default=4)     # labels <= split_index are negative
    p.add_argument("--numGPU", type=int, default=1)          # parsed, never read (as in the reference)
    p.add_argument("--total_iter", type=int, default=2000)
    p.add_argument("--neg_keep_ratio", type=float, default=1)
    p.add_argument("--local_rank", type=int, default=0)
    p.add_argument("--master_addr", type=str)
    p.add_argument("--test_ratio", type=float, default=0.0001)
    # ---- build extras
    p.add_argument("--arch", type=str, default="resnet50")
    p.add_argument("--image_size", type=int, default=128, help="reference resizes to 128x128 (main.py:95)")
    p.add_argument("--synthetic", action="store_true", default=True,
                   help="synthetic on-device ImageNet-shaped data (the only data source offline)")
    p.add_argument("--dataset_size", type=int, default=1281167)
    p.add_argument("--num_classes", type=int, default=1000)
    p.add_argument("--pos_ratio", type=float, default=None,
                   help="synthetic positive fraction; default follows split_index like ImageNet")
    p.add_argument("--partition", choices=["reference", "stratified"], default="stratified",
                   help="reference: data_partitioner.py index lists; stratified: imbalance-preserving shards")
    p.add_argument("--mode", choices=["reference", "paper"], default="reference",
                   help="reference: main.py quirks (b prox uses a, no alpha ascent); paper: intended PPD-SG")
    p.add_argument("--bf16", action=argparse.BooleanOptionalAction, default=True,
                   help="bf16 autocast for the backbone (fp32 master weights and fp32 AUC kernels)")
    p.add_argument("--channels_last", action=argparse.BooleanOptionalAction, default=True)
    p.add_argument("--fused_bn", action=argparse.BooleanOptionalAction, default=True,
                   help="training-mode BatchNorm + residual add + ReLU through the fused HIP kernels "
                        "(needs --channels_last; csrc/bn_act.hip)")
    p.add_argument("--gemm_conv1x1", action=argparse.BooleanOptionalAction, default=True,
                   help="stride-1 1x1 convolutions as hipBLASLt GEMMs where a per-shape timing says so "
                        "(needs --channels_last; conv1x1.py)")
    p.add_argument("--head", choices=["softmax", "logits"], default="softmax",
                   help="softmax: the model ends in Softmax like resnet.py:159; logits: the softmax column is "
                        "folded into the fused surrogate kernel")
    p.add_argument("--split_eval", type=int, default=1,
                   help="1: every rank scores a share of the test set with rank 0's model (the same AUC "
                        "bit for bit only with --deterministic_eval 1; otherwise as close as two rank-0 scorings); "
                        "0: rank 0 scores it all (main.py:232)")
    p.add_argument("--deterministic_eval", type=int, default=0,
                   help="1: score the test set with repeatable convolution solvers (cudnn.deterministic), so "
                        "split and rank-0 scoring give the same bits; MIOpen's deterministic choices for "
                        "ResNet-50 224^2 bf16 are ~100x slower than its default ones")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--history_dir", type=str, default="history")
    p.add_argument("--backend", type=str, default=None, help="torch.distributed backend (default nccl=RCCL)")
    return p


def parse(argv=None) -> argparse.Namespace:
    return get_parser().parse_args(argv)


para = get_parser().parse_args([])
