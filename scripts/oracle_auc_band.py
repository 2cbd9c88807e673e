"""The CPU oracle loop's test AUC at the bench's in-training evaluation point.

bench.py trains ResNet-50 b256 224^2 (bf16 backbone on the GPU) for warmup + steps + the period
sweep's steps on a pool of 4 resident batches, then scores a test set of 8192 images and reports its
exact AUC. This runs the reference's own algorithm on the SAME synthetic data distribution -- the
oracle's restatement of main.py:140-334 (oracle/reference_cpu.train_stage1_world1: the verbatim
loss, autograd, per-tensor dppd_sg, the alpha estimate), fp32 torch on the CPU -- with the same
label sequence, pool, sign flips, lr and step count (only the pixel noise differs: the CPU and the
GPU draw from different generators), then the test AUC with sklearn (main.py:79-81, eval mode). Its
result is the band bench.py reports beside training_eval.auc, with the exact Bayes ceiling of the
test set (loader.signal_auc_ceiling: 1 - flip in expectation). TEST / MEASUREMENT INFRASTRUCTURE:
the oracle is the thing run here, on purpose; nothing of the product path is.

    python scripts/oracle_auc_band.py --steps 153 --seeds 0 --out profiles/r05/oracle_auc_band.json
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--pool", type=int, default=4)
    ap.add_argument("--steps", type=int, default=153, help="bench: warmup 5 + steps 20 + sweep 4 x 32")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--gamma", type=float, default=2000.0)
    ap.add_argument("--pos-ratio", type=float, default=0.1)
    ap.add_argument("--flip", type=float, default=0.2)
    ap.add_argument("--test", type=int, default=8192)
    ap.add_argument("--test-batch", type=int, default=256)
    ap.add_argument("--seeds", default="0", help="extra torch seeds for the init (bench: 1234 + seed)")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)

    from distributedauc_amd.backbone import build_backbone
    from distributedauc_amd.loader import DeviceLoader, SyntheticImageNet, imagenet_like_labels, signal_auc_ceiling
    from oracle import reference_cpu as R

    split = 499
    runs = []
    # the bench's data: training labels of rank 0 (make_coda), the test set of bench_training_eval
    train_labels = imagenet_like_labels(1 << 16, 1000, split, pos_ratio=args.pos_ratio, seed=123)
    test_labels = imagenet_like_labels(args.test, 1000, split, pos_ratio=args.pos_ratio, seed=777)
    ceiling = signal_auc_ceiling(np.arange(args.test), test_labels, split, args.flip)
    for sd in (int(v) for v in args.seeds.split(",")):
        t0 = time.time()
        torch.manual_seed(1234 + sd)
        net = build_backbone(args.arch, num_classes=2).to(memory_format=torch.channels_last)
        ds = SyntheticImageNet(train_labels, args.image_size, split)
        loader = DeviceLoader(ds, np.arange(len(train_labels)), args.batch, "cpu", seed=1234 + sd, channels_last=True,
                              pool=args.pool, flip=args.flip)
        losses, abal = R.train_stage1_world1(net, iter(loader), args.steps, args.lr, args.gamma, split, I=16)
        t1 = time.time()
        tds = SyntheticImageNet(test_labels, args.image_size, split)
        tl = iter(DeviceLoader(tds, np.arange(args.test), args.test_batch, "cpu", seed=777, shuffle=False,
                               channels_last=True, flip=args.flip))
        net.eval()
        scores, labs = [], []
        with torch.no_grad():
            for _ in range((args.test + args.test_batch - 1) // args.test_batch):
                x, lab = next(tl)
                scores.append(net(x)[:, 1].float())
                labs.append(torch.where(lab > split, 1, -1))
        s = torch.cat(scores)[: args.test].numpy()
        y = torch.cat(labs)[: args.test].numpy()
        auc = R.auc_sklearn(y, s)
        runs.append({"seed": 1234 + sd, "test_auc": auc, "final_loss": losses[-1], "a_b_alpha": abal,
                     "train_seconds": t1 - t0, "eval_seconds": time.time() - t1,
                     "losses_every_10": losses[::10]})
        print(json.dumps(runs[-1]), flush=True)
    rec = {"what": "CPU oracle loop (oracle/reference_cpu.train_stage1_world1: main.py:140-334 restated, fp32 "
                   "torch CPU) on bench.py's in-training evaluation workload; test AUC by sklearn",
           "config": {"arch": args.arch, "batch": args.batch, "image_size": args.image_size, "pool": args.pool,
                      "steps": args.steps, "lr": args.lr, "gamma": args.gamma, "pos_ratio": args.pos_ratio,
                      "signal": 0.25, "flip": args.flip, "test_images": args.test, "threads": args.threads},
           "bayes_ceiling_test_set": ceiling, "runs": runs,
           "band": [min(r["test_auc"] for r in runs), max(r["test_auc"] for r in runs)]}
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps({k: rec[k] for k in ("bayes_ceiling_test_set", "band")}))


if __name__ == "__main__":
    main()
