"""The reference's own CoDA loop on the CPU, on the bench's synthetic data: which way does the AUC go?

VERDICT r03 #1 asks what the reference algorithm itself does on this setup. This runs the oracle's
restatement of the reference's op sequence (oracle/reference_cpu.py: the verbatim loss of
main.py:313-317, autograd, per-tensor dppd_sg of main.py:56-64, the alpha estimate of
main.py:166-197 in eval mode) with world 1, fp32 torch CPU, on the data loader.py builds (N(0,1)
pixels, +-signal on channel 0 by class), a pool of cycled training batches as bench.py uses, and
reports the AUC of the training pool and of a test set in eval mode (running BN statistics) and
train mode (batch statistics) at step marks.

    python scripts/cpu_oracle_direction.py --arch resnet18 --image-size 32 --batch 64 --steps 150
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def make_batches(n_batches, B, R, pos_ratio, signal, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n_batches):
        y = torch.where(torch.rand(B, generator=g) < pos_ratio, 1, -1)
        x = torch.randn(B, 3, R, R, generator=g)
        x[:, 0] += signal * y.float().view(-1, 1, 1)
        out.append((x, y))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--image-size", type=int, default=32)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--pool", type=int, default=4)
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--marks", default="0,10,25,50,100,150")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--gamma", type=float, default=2000.0)
    ap.add_argument("--signal", type=float, default=0.25)
    ap.add_argument("--test", type=int, default=2048)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)

    from distributedauc_amd.backbone import build_backbone
    from oracle import reference_cpu as R

    torch.manual_seed(1234)
    net = build_backbone(args.arch, num_classes=2)
    pool = make_batches(args.pool, args.batch, args.image_size, 0.1, args.signal, 123)
    test = make_batches((args.test + 255) // 256, 256, args.image_size, 0.1, args.signal, 777)
    a, b, alpha = (torch.zeros(1, requires_grad=True) for _ in range(3))
    gpos, gneg = torch.zeros(1), torch.zeros(1)

    # stage 1 start (main.py:154-208): anchor, alpha over 3 batches in eval mode
    net0 = {k: v.clone() for k, v in net.state_dict().items()}
    net.eval()
    hn = hp = nn_ = np_ = 0.0
    with torch.no_grad():
        for k in range(3):
            x, y = pool[k % len(pool)]
            h = net(x)[:, 1]
            hn += float((h * (y == -1).float()).sum()); nn_ += float((y == -1).sum())
            hp += float((h * (y == 1).float()).sum()); np_ += float((y == 1).sum())
    net.train()
    alpha.data = torch.tensor([hn / nn_ - hp / np_], dtype=torch.float32)
    a0, b0, alpha0 = a.detach().clone(), b.detach().clone(), alpha.detach().clone()

    def score(batches, mode):
        bufs = [t.clone() for t in net.buffers()]
        net.train(mode == "train")
        hs, ys = [], []
        with torch.no_grad():
            for x, y in batches:
                hs.append(net(x)[:, 1])
                ys.append(y)
        for t, s in zip(net.buffers(), bufs):
            t.copy_(s)
        net.train()
        h, y = torch.cat(hs).numpy().astype(np.float64), torch.cat(ys).numpy()
        return {"auc": R.auc_sklearn(y, h), "mean_pos": float(h[y == 1].mean()), "mean_neg": float(h[y == -1].mean())}

    lpos, lneg = torch.zeros(1), torch.zeros(1)
    recs = []
    t = 0
    for m in sorted({int(v) for v in args.marks.split(",")}):
        while t < m:
            x, y = pool[t % len(pool)]
            lpos += float((y == 1).sum()); lneg += float((y == -1).sum())
            p = torch.tensor([float(gpos + lpos) / float(gpos + lpos + gneg + lneg)])
            h = net(x)[:, 1]
            loss = R.surrogate_loss(h, y, a, b, alpha, p)
            net.zero_grad()
            a.grad = b.grad = alpha.grad = None
            loss.backward()
            with torch.no_grad():
                for name, prm in net.named_parameters():
                    prm.data = R.pd_step(prm.data, prm.grad.data, net0[name], args.lr, args.gamma)
                na, nb, nal = R.scalar_update(float(a), float(b), float(alpha), float(a.grad), float(b.grad),
                                              float(alpha.grad), float(a0), float(b0), float(alpha0), args.lr,
                                              args.gamma)
                a.data.fill_(float(na)); b.data.fill_(float(nb)); alpha.data.fill_(float(nal))
            t += 1
            last = float(loss)
        rec = {"step": t, "loss": last if t else None, "a": float(a), "b": float(b), "alpha": float(alpha),
               "train_eval": score(pool, "eval"), "train_train": score(pool, "train"),
               "test_eval": score(test, "eval"), "test_train": score(test, "train")}
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"args": vars(args), "records": recs}, indent=1))


if __name__ == "__main__":
    main()
