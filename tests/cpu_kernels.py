"""CPU stand-ins for the libdauc.so kernels, built on the oracle (TEST INFRASTRUCTURE).

Used only by the CPU (no-GPU) tests of the host orchestration: the CoDA loop,
its multi-process gloo averaging and the flat-buffer bookkeeping run unchanged
while each ``distributedauc_amd.ops`` call is served by the oracle's restatement
of the same reference lines. The product itself has no CPU path; these
stand-ins are installed only by ``install(monkeypatch)`` inside tests.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from oracle import reference_cpu as R


def label_map_phat(labels, split_index, y_out, lcounts, gcounts, p_hat):
    y = torch.where(labels <= split_index, -1, 1)
    y_out.copy_(y.to(torch.int8))
    lcounts[0] += float((y == 1).sum())
    lcounts[1] += float((y == -1).sum())
    p_hat[0] = float(R.phat(gcounts[0].item(), gcounts[1].item(), lcounts[0].item(), lcounts[1].item()))


def surrogate_fwdbwd(h, y, abalpha, p_hat, *, dh=None, out64=None, grad3=None, loss=None):
    a, b, al = (float(v) for v in abalpha[:3])
    F, dh64, da, db, dal = R.surrogate_closed_form(h.detach().numpy(), y.numpy(), a, b, al, float(p_hat[0]))
    if dh is not None:
        dh.copy_(torch.from_numpy(dh64.astype(np.float32)))
    if out64 is not None:
        out64[:6] = torch.tensor([F, da, db, dal, float((y == 1).sum()), float((y == -1).sum())])
    if grad3 is not None:
        grad3[:3] = torch.tensor([da, db, dal], dtype=torch.float32)
    if loss is not None:
        loss.fill_(float(F))


def class_sums(h, y, sums4, accumulate=True):
    hd = h.detach().double()
    v = torch.tensor([hd[y == -1].sum(), (y == -1).sum(), hd[y == 1].sum(), (y == 1).sum()], dtype=torch.float64)
    if accumulate:
        sums4 += v
    else:
        sums4.copy_(v)


def alpha_from_sums(sums4, alpha):
    s = sums4.tolist()
    alpha[0] = float(np.float32(s[0] / s[1] - s[2] / s[3]))


def coda_finalize(flat, n_avg, world, lcounts, gcounts):
    if world > 1:
        flat[:n_avg] /= float(world)
    gcounts += lcounts
    lcounts.zero_()


def scale_div(x, divisor):
    x /= float(divisor)


def pd_update(w, w0, w_avg, segs, nseg, *, scalars=None, grad3=None, anchor3=None, lr, gamma, mode="reference"):
    """Walks the same segment table the HIP kernel receives (raw host pointers on CPU)."""
    if scalars is not None:
        s = scalars.tolist()
        g = grad3.tolist()
        an = anchor3.tolist()
        scalars[:3] = torch.tensor(R.scalar_update(*s[:3], *g[:3], *an[:3], lr, gamma, mode))
    for i in range(nseg):
        sg = segs[i]
        n, off = sg.numel, sg.offset
        g = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_float * n).from_address(sg.grad)).copy())
        new = R.pd_step(w[off:off + n], g, w0[off:off + n], lr, gamma)
        w[off:off + n] = new
        if w_avg is not None:
            w_avg[off:off + n] += new


def compact_positives(scores, labels):
    """Stable compaction stand-in: (pos buffer of capacity n, stats {P, n - P, non-finite pos, other})."""
    s, y = scores.detach(), labels
    pos = torch.empty_like(s)
    m = y == 1
    P = int(m.sum())
    pos[:P] = s[m]
    other = int(((y != 1) & (y != -1)).sum())
    return pos, torch.tensor([P, s.numel() - P, int((~torch.isfinite(s[m])).sum()), other], dtype=torch.int64)


def auc_counts_sorted_labeled(pos, scores, labels, begin, end, wins_ties, nonfinite=None):
    """(wins, ties) of every label != 1 in [begin, end) against pos, by the C oracle's brute force."""
    neg = scores[begin:end][labels[begin:end] != 1].numpy()
    W, T = coracle_pair_count(pos.numpy(), neg)
    wins_ties[0] += W
    wins_ties[1] += T
    if nonfinite is not None:
        nonfinite[0] += int((~np.isfinite(neg)).sum())


def auc_eval_counts(scores, labels):
    """The one-call evaluation stand-in: (W, T, P, N, non-finite, other) by the C oracle."""
    from oracle import coracle

    s, y = scores.detach().numpy(), labels.numpy().astype(np.int64)
    P = int((y == 1).sum())
    bad = int((~np.isfinite(s)).sum())
    other = int(((y != 1) & (y != -1)).sum())
    if bad or P == 0 or P == s.size:
        return 0, 0, P, s.size - P, bad, other
    e = coracle.auc_counts(np.where(y == 1, 1, -1), s)
    return e["wins"], e["ties"], P, s.size - P, 0, other


def auc_eval_counts_part(scores, labels, part, parts, part_counts):
    """dauc_auc_eval_counts_part's stand-in: every part sees all positives, queries its slice."""
    s, y = scores.detach().numpy(), labels.numpy().astype(np.int64)
    n = s.size
    ispos = y == 1
    P, N = int(ispos.sum()), n - int(ispos.sum())
    other = int(((y != 1) & (y != -1)).sum())
    fin = np.isfinite(s)
    if P <= N:
        bad = int((~fin[ispos]).sum())  # the compaction checks the positives' scores
    else:
        bad = int((~fin).sum())  # the split checks every score
    if bad or P == 0 or N == 0:
        return 0, 0, P, N, bad, other, 0
    pos, negs = s[ispos], s[~ispos]
    if P <= N:
        lo, hi = n * part // parts, n * (part + 1) // parts
        q = s[lo:hi][y[lo:hi] != 1]
        qbad = int((~np.isfinite(q)).sum())
        W, T = coracle_pair_count(pos, q[np.isfinite(q)]) if q.size else (0, 0)
    else:
        lo, hi = P * part // parts, P * (part + 1) // parts
        qbad = 0
        W, T = coracle_pair_count(pos[lo:hi], negs) if hi > lo else (0, 0)
    part_counts[0], part_counts[1], part_counts[2] = W, T, qbad
    return W, T, P, N, bad, other, qbad


def auc_eval_enqueue(scores, labels, part, parts, out=None):
    """dauc_auc_eval_enqueue's stand-in: the part's 8-word record (W, T, #non-finite queried,
    P, 0, #non-finite positives, #labels not in {-1, 1}, verdict). The index holds the table when
    P <= n / 2 + 1 (verdict 1); larger tables get verdict 2 (the blocking sorted path)."""
    s, y = scores.detach().numpy(), labels.numpy().astype(np.int64)
    n = s.size
    ispos = y == 1
    P = int(ispos.sum())
    other = int(((y != 1) & (y != -1)).sum())
    nfpos = int((~np.isfinite(s[ispos])).sum())
    lo, hi = n * part // parts, n * (part + 1) // parts
    rec = torch.zeros(8, dtype=torch.int64) if out is None else out
    rec.zero_()
    rec[3], rec[5], rec[6] = P, nfpos, other
    if hi <= lo:
        return rec
    verdict = 1 if P <= n // 2 + 1 else 2
    rec[7] = verdict
    q = s[lo:hi][y[lo:hi] != 1]
    rec[2] = int((~np.isfinite(q)).sum())
    if verdict == 1 and P and not nfpos:
        W, T = coracle_pair_count(s[ispos], q[np.isfinite(q)]) if q.size else (0, 0)
        rec[0], rec[1] = W, T
    return rec


_INDEX_CAP = 219_838  # 3 / 2 x the count index's cells (auc_sort.hip direct_capacity)


def _slot_cap(parts):
    """auc_eval.hip slot_cap: an even share of the index's capacity + 25 % + 64, whatever n."""
    fair = -(-_INDEX_CAP // parts)
    return fair + fair // 4 + 64


_SLOT_HIST = 256                  # the slot's top-bucket histogram (2048 u32) after the header
_SLOT_HDR = _SLOT_HIST + 2048 * 4  # the slot's scores


def auc_slot_bytes(n, parts):
    """dauc_auc_slot_bytes' stand-in (same formula; n only has to be >= 1)."""
    return _SLOT_HDR + -(-_slot_cap(parts) * 4 // 256) * 256


def _keys(v):
    """count_index.h key_fast: the order-preserving uint32 key (-0 on +0)."""
    u = (np.asarray(v, np.float32) + np.float32(0)).view(np.uint32)
    return u ^ np.where(u >> 31 != 0, np.uint32(0xffffffff), np.uint32(0x80000000))


def _top_buckets(pos):
    """count_index.h's top-bucket histogram of the scores' order-preserving keys (-0 on +0)."""
    return np.bincount(_keys(pos) >> 21, minlength=2048).astype(np.uint32)


def _slice_lo(n, part, parts):
    return 0 if part == 0 else (n if part >= parts else (n * part // parts) & ~255)


def _query_range(n, part, parts):
    """auc_eval.hip query_lo / query_hi: part r counts the NEXT part's slice."""
    q = (part + 1) % parts
    return _slice_lo(n, q, parts), _slice_lo(n, q + 1, parts)


def auc_eval_compact_part(scores, labels, part, parts, slot):
    """dauc_auc_eval_compact_part's stand-in: header {P_r, 0, #non-finite positives, #other labels,
    n} (int64) at byte 0, the positives' top-bucket histogram from byte 256, the slice's positive
    scores (in order) from byte 8448, at most cap of them."""
    s, y = scores.detach().numpy(), labels.numpy().astype(np.int64)
    n = s.size
    lo, hi = _slice_lo(n, part, parts), _slice_lo(n, part + 1, parts)
    ss, yy = s[lo:hi], y[lo:hi]
    pos = ss[yy == 1]
    hdr = np.array([pos.size, 0, int((~np.isfinite(pos)).sum()), int(((yy != 1) & (yy != -1)).sum()), n], np.int64)
    slot[:40] = torch.from_numpy(hdr.view(np.uint8).copy())
    slot[_SLOT_HIST:_SLOT_HDR] = torch.from_numpy(_top_buckets(pos).view(np.uint8).copy())
    k = min(pos.size, _slot_cap(parts))
    slot[_SLOT_HDR:_SLOT_HDR + 4 * k] = torch.from_numpy(pos[:k].astype(np.float32).view(np.uint8).copy())
    return slot


def auc_eval_query_part(scores, labels, part, parts, slots, out=None):
    """dauc_auc_eval_query_part's stand-in: the gathered slots' positives (verdict 2 when a slot
    overflowed or the table exceeds the index), the next part's slice counted, the record's check
    word (low half: the queried slot's P - this rank's positives over that slice, mod 2^32; high
    half: slots built for another n); the enqueue record otherwise."""
    s, y = scores.detach().numpy(), labels.numpy().astype(np.int64)
    n = s.size
    nb, cap = auc_slot_bytes(n, parts), _slot_cap(parts)
    raw = slots.numpy()
    P = nfpos = other = 0
    over = False
    pos = []
    hdrs = []
    for r in range(parts):
        h = raw[r * nb:r * nb + 40].view(np.int64)
        hdrs.append(h)
        P, nfpos, other = P + int(h[0]), nfpos + int(h[2]), other + int(h[3])
        over |= int(h[0]) > cap
        pos.append(raw[r * nb + _SLOT_HDR:r * nb + _SLOT_HDR + 4 * min(int(h[0]), cap)].view(np.float32))
    pos = np.concatenate(pos) if pos else np.zeros(0, np.float32)
    lo, hi = _query_range(n, part, parts)
    rec = torch.zeros(8, dtype=torch.int64) if out is None else out
    rec.zero_()
    rec[3], rec[5], rec[6] = P, nfpos, other
    qh = hdrs[(part + 1) % parts]
    mism = sum(int(h[4]) != n for h in hdrs)
    yq, sq = y[lo:hi], s[lo:hi]
    low = (int(qh[0]) - int((yq == 1).sum())) & 0xFFFFFFFF
    rec[4] = (mism << 32) | low
    if hi <= lo:
        return rec
    verdict = 1 if (not over and 0 < P <= min(n // 2 + 1, _INDEX_CAP)) else 2
    rec[7] = verdict
    q = sq[yq != 1]
    rec[2] = int((~np.isfinite(q)).sum())
    if verdict == 1 and not nfpos:
        W, T = coracle_pair_count(pos, q[np.isfinite(q)]) if q.size else (0, 0)
        rec[0], rec[1] = W, T
    return rec


def split_scores(scores, labels, negatives=True):
    """dauc_split_scores' stand-in: stable (pos, neg) buffers of capacity n and the stats
    {P, N, #non-finite scores, #labels not in {-1, 1}} (N counts every label != 1)."""
    s, y = scores.detach(), labels
    m = y == 1
    P = int(m.sum())
    pos, neg = torch.empty_like(s), torch.empty_like(s) if negatives else None
    pos[:P] = s[m]
    if negatives:
        neg[: s.numel() - P] = s[~m]
    other = int(((y != 1) & (y != -1)).sum())
    return pos, neg, torch.tensor([P, s.numel() - P, int((~torch.isfinite(s)).sum()), other], dtype=torch.int64)


def pair_count(pos, neg, wins_ties, variant=0):
    """dauc_pair_count's stand-in: wins_ties[0:2] += the brute-force (wins, ties) of pos x neg."""
    W, T = coracle_pair_count(pos.detach().numpy(), neg.detach().numpy())
    wins_ties[0] += W
    wins_ties[1] += T


def coracle_pair_count(pos, neg):
    from oracle import coracle

    return coracle.pair_count_bruteforce(pos, neg)


def install(monkeypatch):
    from distributedauc_amd import flat, ops

    for name in ("label_map_phat", "surrogate_fwdbwd", "class_sums", "alpha_from_sums", "coda_finalize",
                 "scale_div", "pd_update", "compact_positives", "auc_counts_sorted_labeled", "auc_eval_counts",
                 "auc_eval_counts_part", "auc_eval_enqueue", "auc_slot_bytes", "auc_eval_compact_part",
                 "auc_eval_query_part", "split_scores", "pair_count"):
        monkeypatch.setattr(ops, name, globals()[name])
    monkeypatch.setattr(flat, "_check_device", lambda dev: None)


class _Patcher:
    """Minimal monkeypatch for spawned worker processes (no pytest fixture there)."""

    def setattr(self, obj, name, value):
        setattr(obj, name, value)


def install_in_process():
    install(_Patcher())
