"""Which way does CoDA training move the AUC, and does eval mode agree with train mode?

VERDICT r03 #1: the bench's in-training test AUC was 0.048 (an inversion). This probe trains the
bench's own CoDA (bench.make_coda: same data, pool, lr, I) and at fixed step marks scores
  - the training pool in eval mode (running BN statistics) and in train mode (batch statistics,
    running statistics saved and restored),
  - the bench's test set the same two ways, eval mode with and without fixed_engine("gemm"),
and reports each AUC from the GPU kernels and from sklearn on the host (the two must agree), plus
the loss, a, b, alpha and the class means of h on the training pool.

    python scripts/diag_auc_direction.py --arch resnet50 --batch 256 --image-size 224 --steps 150
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

from distributedauc_amd import use_tuned_miopen_db  # noqa: E402

use_tuned_miopen_db()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--marks", default="0,10,25,50,100,150")
    ap.add_argument("--pool", type=int, default=4)
    ap.add_argument("--fused-bn", type=int, default=1)
    ap.add_argument("--gemm", type=int, default=1)
    ap.add_argument("--amp", type=int, default=1, help="bf16 autocast backbone (1) or fp32 (0)")
    ap.add_argument("--eval-images", type=int, default=4096)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--I", type=int, default=16)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import bench
    from sklearn.metrics import roc_auc_score

    from distributedauc_amd.auc import AUC
    from distributedauc_amd.conv1x1 import fixed_engine
    from distributedauc_amd.loader import DeviceLoader, SyntheticImageNet, imagenet_like_labels

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    coda, it = bench.make_coda(args.arch, args.batch, args.image_size, args.I, 0.1, args.pool, 1, 0, dev,
                               args.fused_bn, args.gemm)
    coda.lr = coda.lr0 = args.lr
    if not args.amp:
        coda.autocast_dtype = None
    pool = [next(it) for _ in range(args.pool)]  # the cycled training batches, in order

    n = args.eval_images
    tb = args.batch
    tl = imagenet_like_labels(n, 1000, 499, pos_ratio=0.1, seed=777)
    tit = iter(DeviceLoader(SyntheticImageNet(tl, args.image_size, 499), np.arange(n), tb, dev, seed=777,
                            shuffle=False, channels_last=True))
    test = [next(tit) for _ in range((n + tb - 1) // tb)]

    def score(batches, mode, gemm_fixed=True):
        bufs = [b.clone() for b in coda.model.buffers()]
        coda.model.train(mode == "train")
        hs, ys = [], []
        ctx = fixed_engine("gemm") if gemm_fixed else torch.no_grad()
        with torch.no_grad(), ctx:
            for x, lab in batches:
                hs.append(coda.scores(x).float())
                ys.append(torch.where(lab > 499, 1, -1).to(torch.int8))
        with torch.no_grad():
            for b, s in zip(coda.model.buffers(), bufs):
                b.copy_(s)
        coda.model.train()
        h, y = torch.cat(hs), torch.cat(ys)
        gpu = AUC(y, h)
        hh, yy = h.cpu().numpy().astype(np.float64), y.cpu().numpy()
        skl = float(roc_auc_score(yy, hh)) if len(set(yy.tolist())) == 2 else float("nan")
        return {"auc": gpu, "sklearn": skl, "mean_pos": float(hh[yy == 1].mean()),
                "mean_neg": float(hh[yy == -1].mean()), "finite": bool(np.isfinite(hh).all())}

    marks = sorted({int(v) for v in args.marks.split(",")})
    recs = []
    t = 0
    for m in marks:
        while t < m:
            x, y = pool[t % len(pool)]
            coda.train_step(x, y)
            t += 1
        torch.cuda.synchronize()
        ab = coda.state.abalpha.tolist()
        rec = {"step": t, "loss": float(coda.last_loss.item()) if coda.last_loss is not None else None,
               "a": ab[0], "b": ab[1], "alpha": ab[2], "p_hat": float(coda.state.p_hat.item()),
               "train_eval": score(pool, "eval"), "train_train": score(pool, "train"),
               "test_eval": score(test, "eval"), "test_eval_nofix": score(test, "eval", gemm_fixed=False),
               "test_train": score(test, "train")}
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    out = {"args": vars(args), "records": recs, "time": time.strftime("%Y-%m-%d %H:%M:%S")}
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
