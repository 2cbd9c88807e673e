"""CPU restatement of the reference's data-parallel AUC hot path.

TEST INFRASTRUCTURE ONLY. Nothing in the product (``distributedauc_amd``)
imports this module. It is used solely by ``tests/``, by
``__graft_entry__.smoke()`` and by ``bench.py``'s ``cpu_baseline`` leg, as the
checker the HIP path is compared against and as the timed CPU path.

Each function restates one piece of ZhishuaiGuo/DistributedAUC
(``/root/reference/imagenet``) and cites the file:line it follows. The
restatement is pinned against the reference itself: ``tests/golden/make_golden.py``
imported the reference in the build container (torchvision stubbed) and froze
its outputs as fixtures under ``tests/golden/``; ``tests/test_oracle_golden.py``
checks every function here against those fixtures.

Exact-AUC arithmetic lives in scikit-learn (third party, absent from the
reference tree; sklearn 1.7.2 in this image). ``auc_sklearn`` calls it exactly
as main.py:79-81 does; ``auc_counts`` restates sklearn's ``_binary_clf_curve``
(sklearn/metrics/_ranking.py:826-908) to recover the integer counts.
"""
from __future__ import annotations

import random
import warnings

import numpy as np
import torch

__all__ = [
    "label_map",
    "phat",
    "surrogate_loss",
    "surrogate_fwdbwd_fp32",
    "surrogate_closed_form",
    "pd_step",
    "dppd_sg_flat",
    "scalar_update",
    "coda_average",
    "auc_sklearn",
    "auc_counts",
    "auc_from_counts",
    "partition_indices",
    "alpha_from_sums",
]


# --------------------------------------------------------------- a1 (main.py:303-310)
def label_map(labels: np.ndarray, split_index: int) -> np.ndarray:
    """main.py:303-304: class index <= split_index -> -1, else +1."""
    labels = np.asarray(labels)
    return np.where(labels <= split_index, -1, 1).astype(np.int64)


def phat(gpos: float, gneg: float, lpos: float, lneg: float) -> np.float32:
    """main.py:309-310.

    ``global_total_*`` are fp32 tensors; the sums are fp32 tensor adds, ``float()``
    turns them into Python doubles, the ratio is a double divide and the result
    lands in an fp32 tensor (``p_hat*0 + ratio``).
    """
    f = np.float32
    num = f(f(gpos) + f(lpos))
    den = f(f(f(num) + f(gneg)) + f(lneg))
    return np.float32(float(num) / float(den))


# --------------------------------------------------------------- a2/a3 (main.py:311-326)
def surrogate_loss(h: torch.Tensor, y: torch.Tensor, a, b, alpha, p) -> torch.Tensor:
    """The inline loss of main.py:313-317, same operations in the same order.

    ``h`` is the positive-class score, ``y`` holds +1/-1, means divide by B.
    """
    pos = (1 == y).float()
    neg = (-1 == y).float()
    term_pos = (1 - p) * torch.mean((h - a) ** 2 * pos)
    term_neg = p * torch.mean((h - b) ** 2 * neg)
    term_cross = 2 * (1 + alpha) * torch.mean((p * h * neg - (1 - p) * h * pos))
    return term_pos + term_neg + term_cross - p * (1 - p) * (alpha ** 2)


def surrogate_fwdbwd_fp32(h, y, a, b, alpha, p):
    """torch-fp32 autograd of the reference loss (main.py:313-317 + backward at 326).

    Returns (F, dF/dh, dF/da, dF/db, dF/dalpha) as float32 numpy values.
    """
    ht = torch.tensor(np.asarray(h, np.float32), requires_grad=True)
    yt = torch.tensor(np.asarray(y, np.int64))
    at = torch.tensor([np.float32(a)], requires_grad=True)
    bt = torch.tensor([np.float32(b)], requires_grad=True)
    alt = torch.tensor([np.float32(alpha)], requires_grad=True)
    pt = torch.tensor([np.float32(p)])
    F = surrogate_loss(ht, yt, at, bt, alt, pt)
    F.backward()
    return (
        F.detach().numpy().reshape(-1)[0],
        ht.grad.numpy().copy(),
        at.grad.numpy()[0],
        bt.grad.numpy()[0],
        alt.grad.numpy()[0],
    )


def surrogate_closed_form(h, y, a, b, alpha, p):
    """fp64 closed form of the same loss and gradients."""
    h = np.asarray(h, np.float64)
    y = np.asarray(y)
    B = h.shape[0]
    a, b, alpha, p = (float(np.float32(v)) for v in (a, b, alpha, p))
    pos = (y == 1).astype(np.float64)
    neg = (y == -1).astype(np.float64)
    q = 1.0 - p
    cross = np.sum(p * h * neg - q * h * pos)
    F = (q * np.sum((h - a) ** 2 * pos) + p * np.sum((h - b) ** 2 * neg) + 2 * (1 + alpha) * cross) / B \
        - p * q * alpha ** 2
    dh = (2.0 / B) * (q * (h - a) * pos + p * (h - b) * neg + (1 + alpha) * (p * neg - q * pos))
    da = -2.0 * q * np.sum((h - a) * pos) / B
    db = -2.0 * p * np.sum((h - b) * neg) / B
    dal = 2.0 * cross / B - 2.0 * p * q * alpha
    return F, dh, da, db, dal


# --------------------------------------------------------------- a4/a5 (main.py:56-64, 333-334)
def pd_step(w: torch.Tensor, g: torch.Tensor, w0: torch.Tensor, lr: float, gamma: float) -> torch.Tensor:
    """main.py:61: ``param.data - lr*(param.grad.data + 1/gamma*(param.data - model0[name]))``."""
    return w - lr * (g + 1 / gamma * (w - w0))


def dppd_sg_flat(w, g, w0, lr, gamma, avg=None):
    """dppd_sg over one fp32 vector, plus the running-average add of main.py:333-334.

    Uses torch-CPU fp32 ops in the reference order, so every op is separately
    rounded exactly as the reference's tensors are.
    """
    wt = torch.as_tensor(np.asarray(w, np.float32))
    out = pd_step(wt, torch.as_tensor(np.asarray(g, np.float32)),
                  torch.as_tensor(np.asarray(w0, np.float32)), lr, gamma).numpy()
    if avg is None:
        return out
    return out, (torch.as_tensor(np.asarray(avg, np.float32)) + torch.as_tensor(out)).numpy()


def scalar_update(a, b, alpha, da, db, dalpha, a0, b0, alpha0, lr, gamma, mode: str = "reference"):
    """main.py:58-59 and 64 on the scalars.

    reference mode: b's proximal term uses the updated ``a`` (main.py:59) and the
    dual step only rebinds a local name (main.py:64), so alpha is unchanged.
    paper mode: ``(b - b0)`` and alpha <- alpha + lr*dF/dalpha.
    """
    t = lambda v: torch.tensor([np.float32(v)])  # noqa: E731
    a_t, b_t, al_t = t(a), t(b), t(alpha)
    a_new = a_t - lr * (t(da) + 1 / gamma * (a_t - t(a0)))
    if mode == "reference":
        b_new = b_t - lr * (t(db) + 1 / gamma * (a_new - t(a0)))
        al_new = al_t
    else:
        b_new = b_t - lr * (t(db) + 1 / gamma * (b_t - t(b0)))
        al_new = al_t + lr * t(dalpha)
    return a_new.numpy()[0], b_new.numpy()[0], al_new.numpy()[0]


# --------------------------------------------------------------- a6 (main.py:33-54)
def coda_average(per_rank: list[np.ndarray]) -> np.ndarray:
    """all_reduce(SUM) then ``/= size`` (main.py:37-38, 43-45, 52-54), fp32, rank order."""
    acc = torch.as_tensor(np.asarray(per_rank[0], np.float32)).clone()
    for x in per_rank[1:]:
        acc += torch.as_tensor(np.asarray(x, np.float32))
    acc /= float(len(per_rank))
    return acc.numpy()


def average_all_dist(model, a, b, alpha, gpos, gneg, lpos, lneg, world: int) -> None:
    """main.py:33-54 over a live torch.distributed group (gloo on the CPU baseline):
    one blocking all_reduce(SUM) + ``/= size`` per parameter tensor (buffers untouched,
    main.py:35-38), then a, b, alpha and the local counts (43-47), the global counts
    accumulate the summed locals (49-50), and a, b, alpha are divided (52-54). The caller
    zeroes the locals afterwards (main.py:300-301)."""
    import torch.distributed as dist

    for param in model.parameters():
        dist.all_reduce(param.data, op=dist.ReduceOp.SUM)
        param.data /= float(world)
    for t in (a, b, alpha, lpos, lneg):
        dist.all_reduce(t.data, op=dist.ReduceOp.SUM)
    gpos += lpos
    gneg += lneg
    for t in (a, b, alpha):
        t.data /= float(world)


def alpha_from_sums(h_neg, n_neg, h_pos, n_pos) -> np.float32:
    """main.py:197: ``alpha = h_neg/N_neg - h_pos/N_pos``."""
    return np.float32(h_neg / n_neg - h_pos / n_pos)


# --------------------------------------------------------------- a8 (main.py:79-81)
def auc_sklearn(labels, scores) -> float:
    """main.py:79-81 verbatim in behaviour: sklearn roc_curve(pos_label=1) + auc."""
    from sklearn import metrics

    fpr, tpr, _ = metrics.roc_curve(np.asarray(labels), np.asarray(scores), pos_label=1)
    return float(metrics.auc(fpr, tpr))


def auc_counts(labels, scores) -> dict:
    """Integer AUC counts, restating sklearn/metrics/_ranking.py:826-908.

    _binary_clf_curve sorts scores descending with a stable mergesort (:886),
    keeps the last index of every distinct score (:897), accumulates true
    positives (:901) and derives false positives as ``1 + idx - tps`` (:907).
    From those cumulative counts, per distinct-score group k with dp_k positives
    and dn_k negatives:
        W = sum_k dp_k * (N - fps_k)        (negatives strictly below)
        T = sum_k dp_k * dn_k               (negatives tied)
        2U = sum_k (fps_k - fps_{k-1}) * (tps_k + tps_{k-1})   (sklearn's trapezoid x 2PN)
    and 2U == 2W + T.
    """
    y = np.asarray(labels).reshape(-1) == 1
    s = np.asarray(scores, dtype=np.float32).reshape(-1)
    if not np.all(np.isfinite(s)):
        raise ValueError("Input contains NaN or infinity.")
    order = np.argsort(s, kind="mergesort")[::-1]
    s_sorted = s[order]
    y_sorted = y[order].astype(np.int64)
    distinct = np.where(np.diff(s_sorted))[0]
    thr_idx = np.r_[distinct, y_sorted.size - 1]
    tps = np.cumsum(y_sorted)[thr_idx]
    fps = 1 + thr_idx - tps
    P = int(y.sum())
    N = int(y.size - P)
    tps0 = np.r_[0, tps]
    fps0 = np.r_[0, fps]
    dp = np.diff(tps0)
    dn = np.diff(fps0)
    W = int(np.sum(dp.astype(object) * (N - fps).astype(object)))
    T = int(np.sum(dp.astype(object) * dn.astype(object)))
    two_u = int(np.sum(dn.astype(object) * (tps0[1:] + tps0[:-1]).astype(object)))
    return {"wins": W, "ties": T, "P": P, "N": N, "two_u": two_u}


def auc_from_counts(wins: int, ties: int, P: int, N: int) -> float:
    """(2W + T) / (2PN) in float64; NaN when a class is empty (sklearn warns and returns NaN)."""
    if P == 0 or N == 0:
        warnings.warn("Only one class present in y_true. ROC AUC score is not defined.")
        return float("nan")
    return (2 * wins + ties) / (2 * P * N)


# --------------------------------------------------------------- a9 (data_partitioner.py:19-90)
IMAGENET_NEG = (0, 642289)       # data_partitioner.py:46 -> np.arange(642289)
IMAGENET_POS = (642290, 1281167)  # data_partitioner.py:47 -> np.arange(642290, 1281167)


def partition_indices(sizes, seed: int = 123, neg_keep_ratio: float = 1.0,
                      neg_range=IMAGENET_NEG, pos_range=IMAGENET_POS) -> list[list[int]]:
    """data_partitioner.py:22-90: the reference's index lists, bit for bit.

    The shuffles are Python ``random.Random(seed)`` shuffles of plain lists, so
    the permutation depends only on the list lengths and the call order:
    positives, negatives, then the concatenation ``pos + kept_neg``.
    """
    rng = random.Random()
    rng.seed(seed)
    neg = list(range(*neg_range))
    pos = list(range(*pos_range))
    rng.shuffle(pos)
    rng.shuffle(neg)
    neg = neg[: int(len(neg) * neg_keep_ratio)]
    idx = pos + neg
    rng.shuffle(idx)
    out = []
    n = len(idx)
    for frac in sizes:
        k = int(frac * n)
        out.append(idx[:k])
        idx = idx[k:]
    return out


# --------------------------------------------------------------- the loop (main.py:140-334, size == 1)
def train_stage1_world1(net, batches, steps: int, lr: float, gamma: float, split_index: int, I: int = 16):
    """One rank's stage 1 of the reference's training loop, restated with the functions above.

    main.py:141-142 the pre-training average (size == 1: nothing to average; the counts fold);
    main.py:154-158 the anchor; main.py:170-197 alpha over 3 batches of ``batches`` in eval mode
    (the reference forwards each batch twice, 185 and 187; under no_grad in eval mode both
    passes give the same scores, so one is taken); main.py:210-327 ``steps`` training steps:
    the count fold every I steps (297-301), the label map and counts (303-308), p_hat (309-310),
    the verbatim loss (313-317), zero_grad + backward (318-326) and dppd_sg (327, reference
    quirks). ``batches`` yields CPU (x, class-label) pairs and is consumed exactly as the
    reference consumes ``train_iter``. Returns the per-step losses; ``net`` is trained in place
    and (a, b, alpha) are returned with them."""
    gpos, gneg = torch.zeros(1), torch.zeros(1)
    lpos, lneg = torch.zeros(1), torch.zeros(1)
    a, b, alpha = (torch.zeros(1, requires_grad=True) for _ in range(3))
    net0 = {k: v.clone() for k, v in net.state_dict().items()}
    a0, b0 = a.detach().clone(), b.detach().clone()
    sums = [0.0, 0.0, 0.0, 0.0]
    net.eval()
    with torch.no_grad():
        for _ in range(3):
            x, lab = next(batches)
            y = torch.where(lab <= split_index, -1, 1)
            h = net(x)[:, 1]
            sums[0] += float(torch.sum(h * (y == -1).float()))
            sums[1] += float(torch.sum(y == -1))
            sums[2] += float(torch.sum(h * (y == 1).float()))
            sums[3] += float(torch.sum(y == 1))
    net.train()
    alpha.data = torch.tensor([alpha_from_sums(*sums)], dtype=torch.float32)
    alpha0 = alpha.detach().clone()
    losses = []
    for t_total in range(1, steps + 1):
        x, lab = next(batches)
        if t_total % I == 0:
            gneg += lneg
            gpos += lpos
            lpos, lneg = torch.zeros(1), torch.zeros(1)
        y = torch.where(lab <= split_index, -1, 1)
        lpos += float(torch.sum(y == 1))
        lneg += float(torch.sum(y == -1))
        p = torch.tensor([float(phat(float(gpos), float(gneg), float(lpos), float(lneg)))])
        h = net(x)[:, 1]
        loss = surrogate_loss(h, y, a, b, alpha, p)
        net.zero_grad()
        a.grad = b.grad = alpha.grad = None
        loss.backward()
        with torch.no_grad():
            for name, prm in net.named_parameters():
                prm.data = pd_step(prm.data, prm.grad.data, net0[name], lr, gamma)
            na, nb, nal = scalar_update(float(a), float(b), float(alpha), float(a.grad), float(b.grad),
                                        float(alpha.grad), float(a0), float(b0), float(alpha0), lr, gamma)
            a.data.fill_(float(na))
            b.data.fill_(float(nb))
            alpha.data.fill_(float(nal))
        losses.append(float(loss.detach()))
    return losses, (float(a), float(b), float(alpha))
