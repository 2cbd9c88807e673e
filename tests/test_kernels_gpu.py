"""Parity of every HIP kernel against the CPU oracle and the reference's golden vectors.

Tolerances (fp32 path, north_star: "within 1e-5 relative (fp32)"):
  * surrogate F and scalar gradients: |got - ref| <= 1e-5 * scale, where scale is the
    sum of magnitudes of the terms that make up the value (a plain relative bound
    is meaningless when terms cancel to ~0); against the fp64 closed form 1e-6.
  * dF/dh per element: |got - ref| <= 1e-5 * max(|ref|, c) with c = 2/B * (|h|+|k|) the
    magnitude of the element's factors.
  * update kernel, finalise, stage divide, label map / p_hat: bit-exact.
  * AUC pair counts: bit-exact integers.
"""
from __future__ import annotations

import warnings

import numpy as np
import pytest
import torch

from oracle import coracle
from oracle import reference_cpu as R

pytestmark = pytest.mark.gpu


def T(a, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t if dtype is None else t.to(dtype)


# ------------------------------------------------------------------ surrogate
def _scales(h, y, a, b, al, p):
    h = np.asarray(h, np.float64)
    B = h.size
    pos = (y == 1)
    neg = (y == -1)
    q = 1 - p
    sF = (q * np.sum((h - a) ** 2 * pos) + p * np.sum((h - b) ** 2 * neg)
          + 2 * abs(1 + al) * np.sum(p * h * neg + q * h * pos)) / B + abs(p * q * al * al)
    sa = 2 * q * np.sum(np.abs(h - a) * pos) / B
    sb = 2 * p * np.sum(np.abs(h - b) * neg) / B
    sal = 2 * np.sum(p * h * neg + q * h * pos) / B + abs(2 * p * q * al)
    return np.array([sF, sa, sb, sal])


def _run_surrogate(ops, dev, h, y, abap, h_stride=1, ydtype=torch.int8):
    B = h.size
    if h_stride == 1:
        th = T(h, dev)
    else:
        big = np.zeros((B, h_stride), np.float32)
        big[:, 1] = h
        th = T(big, dev)[:, 1]
    ty = T(y, dev).to(ydtype)
    out64 = torch.zeros(6, dtype=torch.float64, device=dev)
    grad3 = torch.zeros(3, device=dev)
    loss = torch.zeros((), device=dev)
    dh = torch.empty(B, device=dev)
    ops.surrogate_fwdbwd(th, ty, T(abap[:3], dev), T(abap[3:4], dev), dh=dh, out64=out64, grad3=grad3,
                         loss=loss)
    return out64.cpu().numpy(), dh.cpu().numpy(), grad3.cpu().numpy(), loss.item()


def test_surrogate_golden(dev, golden):
    from distributedauc_amd import ops

    z = np.load(golden / "surrogate_cases.npz")
    for ci in range(int(z["ncases"])):
        h, y, abap = z[f"c{ci}_h"], z[f"c{ci}_y"].astype(np.int64), z[f"c{ci}_abap"]
        out64, dh, g3, loss = _run_surrogate(ops, dev, h, y, abap)
        ref32, ref64 = z[f"c{ci}_fp32"].astype(np.float64), z[f"c{ci}_fp64"]
        sc = _scales(h, y, *abap.astype(np.float64))
        assert np.all(np.abs(out64[:4] - ref32) <= 1e-5 * sc + 1e-12), (ci, out64[:4], ref32)
        assert np.all(np.abs(out64[:4] - ref64) <= 1e-6 * sc + 1e-12), (ci, out64[:4], ref64)
        assert np.all(np.abs(g3 - ref32[1:]) <= 1e-5 * sc[1:] + 1e-12)
        assert abs(loss - ref32[0]) <= 1e-5 * sc[0] + 1e-12
        assert out64[4] == np.sum(y == 1) and out64[5] == np.sum(y == -1)
        a, b, al, p = abap.astype(np.float64)
        k = np.where(y == 1, a + 1 + al, b - 1 - al)
        c = 2.0 / h.size * (np.abs(h) + np.abs(k))
        dref = z[f"c{ci}_dh32"].astype(np.float64)
        assert np.all(np.abs(dh - dref) <= 1e-5 * np.maximum(np.abs(dref), c)), ci


@pytest.mark.parametrize("ydtype", [torch.int8, torch.int32, torch.int64])
@pytest.mark.parametrize("stride", [1, 2, 3])
def test_surrogate_strides_and_label_types(dev, ydtype, stride):
    from distributedauc_amd import ops

    rng = np.random.default_rng(stride)
    for B in (1, 255, 256, 1023, 5000, 70_001):
        h = rng.random(B, dtype=np.float32)
        y = np.where(rng.random(B) < 0.2, 1, -1).astype(np.int64)
        y[rng.random(B) < 0.05] = 0
        abap = np.array([0.2, -0.3, 0.05, 0.21], np.float32)
        out64, dh, _, _ = _run_surrogate(ops, dev, h, y, abap, stride, ydtype)
        F, dh64, da, db, dal = R.surrogate_closed_form(h, y, *abap)
        sc = _scales(h, y, *abap.astype(np.float64))
        assert np.all(np.abs(out64[:4] - [F, da, db, dal]) <= 1e-6 * sc + 1e-12), (B, stride)
        k = np.where(y == 1, 0.2 + 1 + 0.05, -0.3 - 1 - 0.05)
        c = 2.0 / B * (np.abs(h) + np.abs(k))
        assert np.all(np.abs(dh - dh64) <= 1e-6 * np.maximum(np.abs(dh64), c))
        assert np.all(dh[y == 0] == 0)


def test_surrogate_large_deterministic(dev):
    """Multi-block path (last-arriver reduce) at 2^24: fp64 closed form + bitwise run-to-run."""
    from distributedauc_amd import ops

    B = 1 << 24
    g = torch.Generator(device=dev).manual_seed(3)
    h = torch.rand(B, device=dev, generator=g)
    y = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
    abap = torch.tensor([0.1, -0.2, 0.3, 0.1], device=dev)
    outs = []
    for _ in range(3):
        o = torch.zeros(6, dtype=torch.float64, device=dev)
        ops.surrogate_fwdbwd(h, y, abap[:3], abap[3:], out64=o)
        outs.append(o.cpu().numpy())
    assert all(np.array_equal(outs[0], o) for o in outs[1:])
    hn, yn = h.cpu().numpy(), y.cpu().numpy().astype(np.int64)
    F, _, da, db, dal = R.surrogate_closed_form(hn, yn, 0.1, -0.2, 0.3, 0.1)
    sc = _scales(hn, yn, 0.1, -0.2, 0.3, float(np.float32(0.1)))
    assert np.all(np.abs(outs[0][:4] - [F, da, db, dal]) <= 1e-6 * sc + 1e-12)
    assert outs[0][4] == np.sum(yn == 1)


@pytest.mark.parametrize("B", [(1 << 20), (1 << 22), (1 << 22) + 37, 3 * (1 << 22) + 4099, (1 << 24) + 5])
def test_surrogate_chunked_variants(dev, B):
    """The one-launch tail kernel (the default for unit-stride B >= 2^22, the extra-reducer kernel)
    and the tuning build's alternatives (include/dauc_tuning.h: 1 persistent, 2 two-launch, 3
    stream alone, 20 the product's kernel at any B, 22 its stream without the reduce): fp64 closed
    form within 1e-6 of term scale, dh and counts bitwise equal across variants (dh is per-element;
    the sums only differ in tree order), bitwise run-to-run, ragged last chunk; the default and the
    variants interleave on one workspace (the epoch-tagged granules need no cleanup between calls)."""
    from distributedauc_amd import ops

    g = torch.Generator(device=dev).manual_seed(B & 0xFFFF)
    h = torch.rand(B, device=dev, generator=g)
    y = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
    y[::97] = 0  # neither class
    abap = torch.tensor([0.1, -0.2, 0.3, 0.1], device=dev)
    hn, yn = h.cpu().numpy(), y.cpu().numpy().astype(np.int64)
    F, dh64, da, db, dal = R.surrogate_closed_form(hn, yn, 0.1, -0.2, 0.3, float(np.float32(0.1)))
    sc = _scales(hn, yn, 0.1, -0.2, 0.3, float(np.float32(0.1)))
    k = np.where(yn == 1, 0.1 + 1 + 0.3, -0.2 - 1 - 0.3)
    c = 2.0 / B * (np.abs(hn) + np.abs(k))
    ref_dh = None
    seen = {}
    for variant in (0, 0, 1, 2, 3, 0, 22, 0, 20, 20, 2, 0, 1, 22, 22, 20, 3, 0, 20):
        o = torch.zeros(6, dtype=torch.float64, device=dev)
        dh = torch.full((B,), float("nan"), device=dev)
        ops.surrogate_fwdbwd(h, y, abap[:3], abap[3:], dh=dh, out64=o, variant=variant)
        got, dhn = o.cpu().numpy(), dh.cpu().numpy()
        if ref_dh is None:
            ref_dh = dhn
        assert np.array_equal(dhn, ref_dh), variant
        assert np.all(np.abs(dhn - dh64) <= 1e-6 * np.maximum(np.abs(dh64), c)), variant
        if variant in (3, 22):  # the stream without its reduce: no scalar outputs
            assert not o.any(), variant
            continue
        assert np.all(np.abs(got[:4] - [F, da, db, dal]) <= 1e-6 * sc + 1e-12), (variant, got, F)
        assert got[4] == np.sum(yn == 1) and got[5] == np.sum(yn == -1), variant
        # fixed summation orders: bitwise run-to-run per kernel (the product at B >= 2^22 is
        # variant 20's kernel)
        key = 20 if variant == 0 and B >= (1 << 22) else variant
        assert np.array_equal(got, seen.setdefault(key, got)), variant
    sums = torch.zeros(4, dtype=torch.float64, device=dev)
    ops.class_sums(h, y, sums, accumulate=False)  # chunked CLASS_ONLY path
    s = sums.cpu().numpy()
    hd = hn.astype(np.float64)
    assert np.allclose(s, [hd[yn == -1].sum(), (yn == -1).sum(), hd[yn == 1].sum(), (yn == 1).sum()],
                       rtol=1e-7, atol=0)


def test_surrogate_tail_ignores_stale_granules(dev):
    """The one-launch loss hands rows over as epoch-tagged granules (surrogate.hip, tail_x kernel):
    a granule written by a workgroup of an EARLIER call -- e.g. one that stored its row after that
    call's reducer gave up waiting -- carries an older tag and is never taken for a current one.
    Here every row and group-total granule of the workspace is overwritten between calls with the
    previous call's tag (and, once, with random tags) and garbage payloads: the next call is
    bit-identical to a clean one, and the epoch word advances by one per call."""
    from distributedauc_amd import _lib, ops

    B = (1 << 22) + 4099
    g = torch.Generator(device=dev).manual_seed(11)
    h = torch.rand(B, device=dev, generator=g)
    y = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
    abap = torch.tensor([0.1, -0.2, 0.3, 0.1], device=dev)

    def call():
        o = torch.zeros(6, dtype=torch.float64, device=dev)
        ops.surrogate_fwdbwd(h, y, abap[:3], abap[3:], out64=o)
        torch.cuda.synchronize()
        return o.cpu().numpy()

    ref = call()
    ws = ops.workspaces.get(dev, "surrogate", _lib.load().dauc_surrogate_workspace_size(B))
    # the tail region's offset (surrogate.hip: tail_offset): the persistent kernel's region
    # (256 + 2048 * 6 * 8 B), then the two-launch form's rows + reduce slots, 256-B aligned
    nb = -(-B // 4096)
    chunk = nb * 48 + 256 + -(-nb // 512) * 48
    off = 256 + 2048 * 48 + -(-chunk // 256) * 256
    gran = ws[off + 256: off + 256 + (nb + 128) * 80].view(torch.int64)  # rows + the 128 reducers' totals
    ew = ws[128:136].view(torch.int64)  # the epoch word: a fixed offset of the workspace (kEpochOffset)
    epoch = int(ew.item()) & 0xFFFFFFFF
    rng = torch.Generator(device=dev).manual_seed(5)
    for k in range(3):
        assert int(ew.item()) & 0xFFFFFFFF == epoch
        garbage = torch.randint(0, 1 << 31, gran.shape, device=dev, generator=rng)
        if k < 2:
            stale_tag = ((epoch - 1) & 0xFFFFFFFF) | 0x80000000
            hi = (stale_tag << 32) - (1 << 64)  # the tag in the high word, as a signed int64
            gran.copy_(garbage + hi)
        else:
            gran.copy_(garbage * (1 << 32) + garbage)  # random tags (bit 31 clear: never current)
        assert np.array_equal(call(), ref), k
        epoch = (epoch + 1) & 0xFFFFFFFF


def test_surrogate_tail_alternating_batch_sizes(dev):
    """The tail kernel's epoch word sits at a fixed offset of the workspace, not in its B-dependent
    tail region: one stream alternating two batch sizes >= 2^22 on one workspace --
    each size's rows where the other size's epoch word used to be -- gives every call bit-identical
    results to its first one, the epoch advances by exactly one per call, and the results match
    the fp64 closed form."""
    from distributedauc_amd import _lib, ops

    sizes = (3 * (1 << 22) + 4099, (1 << 22) + 37, 5 * (1 << 22) + 1)
    g = torch.Generator(device=dev).manual_seed(31)
    data = {}
    for B in sizes:
        h = torch.rand(B, device=dev, generator=g) * 2.0 - 0.5
        y = torch.where(torch.rand(B, device=dev, generator=g) < 0.2, 1, -1).to(torch.int8)
        data[B] = (h, y)
    abap = torch.tensor([0.1, -0.2, 0.3, 0.1], device=dev)
    ws = ops.workspaces.get(dev, "surrogate", max(_lib.load().dauc_surrogate_workspace_size(B) for B in sizes))
    ew = ws[128:136].view(torch.int64)

    def call(B):
        o = torch.zeros(6, dtype=torch.float64, device=dev)
        ops.surrogate_fwdbwd(*data[B], abap[:3], abap[3:], out64=o)
        torch.cuda.synchronize()
        return o.cpu().numpy()

    first = {}
    for i, B in enumerate(sizes * 4 + sizes[::-1] * 2):
        e0 = int(ew.item()) & 0xFFFFFFFF
        got = call(B)
        assert int(ew.item()) & 0xFFFFFFFF == (e0 + 1) & 0xFFFFFFFF, (i, B)
        assert np.array_equal(got, first.setdefault(B, got)), (i, B)
    for B in sizes:
        hn, yn = data[B][0].cpu().numpy(), data[B][1].cpu().numpy().astype(np.int64)
        F, _, da, db, dal = R.surrogate_closed_form(hn, yn, 0.1, -0.2, 0.3, float(np.float32(0.1)))
        sc = _scales(hn, yn, 0.1, -0.2, 0.3, float(np.float32(0.1)))
        assert np.all(np.abs(first[B][:4] - [F, da, db, dal]) <= 1e-6 * sc + 1e-12), B
        assert first[B][4] == np.sum(yn == 1) and first[B][5] == np.sum(yn == -1)


@pytest.mark.timeout(120)
def test_surrogate_timeout_reports_status(dev):
    """a reducer of the one-launch loss that gives up waiting (tuning variant 23:
    one streaming workgroup never publishes its row; the bounded poll takes seconds) makes that
    call's outputs NaN AND sets the workspace's sticky status bit, which dauc_surrogate_status
    reports (ops.surrogate_status: the value, or DaucError with raise_on_error) and clears; a good
    call on the same workspace before and after is exact with status 0."""
    from distributedauc_amd import _lib, ops

    B = 1 << 22
    g = torch.Generator(device=dev).manual_seed(11)
    h = torch.rand(B, device=dev, generator=g)
    y = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
    ab, p = torch.tensor([0.1, -0.2, 0.3], device=dev), torch.tensor([0.1], device=dev)

    def call(variant):
        out64 = torch.zeros(6, dtype=torch.float64, device=dev)
        dh = torch.empty(B, device=dev)
        ops.surrogate_fwdbwd(h, y, ab, p, dh=dh, out64=out64, variant=variant)
        return out64.cpu().numpy(), dh

    good, dh0 = call(20)
    assert np.isfinite(good).all() and ops.surrogate_status(dev, variant=20) == 0
    bad, _ = call(23)
    assert np.isnan(bad[:4]).all(), bad
    assert ops.surrogate_status(dev, variant=20, clear=False) == ops.SURROGATE_TIMEOUT  # sticky
    with pytest.raises(_lib.DaucError, match="timed out"):
        ops.surrogate_status(dev, variant=20, raise_on_error=True)  # reads and clears
    assert ops.surrogate_status(dev, variant=20) == 0
    again, dh1 = call(20)
    assert np.array_equal(again, good) and torch.equal(dh0, dh1)
    assert ops.surrogate_status(dev, variant=20) == 0
    # the product library's own workspace: a clean run reports 0
    ops.surrogate_fwdbwd(h, y, ab, p, out64=torch.zeros(6, dtype=torch.float64, device=dev))
    assert ops.surrogate_status(dev, raise_on_error=True) == 0


def test_surrogate_timing_variants_leave_no_current_rows(dev):
    """The tuning build's stream-only variant of the tail kernel (22) stores its rows but
    reduce nothing, so the epoch does not advance: their rows carry a tag no call expects. A
    product call on OTHER data right after one is bit-identical to the same call after a product
    call (a stale row taken for a current one would change the sums)."""
    from distributedauc_amd import ops

    B = (1 << 22) + 4099
    g = torch.Generator(device=dev).manual_seed(23)
    h1, h2 = torch.rand(B, device=dev, generator=g), torch.rand(B, device=dev, generator=g) * 3.0 - 1.0
    y1 = torch.where(torch.rand(B, device=dev, generator=g) < 0.1, 1, -1).to(torch.int8)
    y2 = torch.where(torch.rand(B, device=dev, generator=g) < 0.4, 1, -1).to(torch.int8)
    abap = torch.tensor([0.1, -0.2, 0.3, 0.1], device=dev)

    def call(h, y, variant=0):
        o = torch.zeros(6, dtype=torch.float64, device=dev)
        ops.surrogate_fwdbwd(h, y, abap[:3], abap[3:], out64=o, variant=variant)
        torch.cuda.synchronize()
        return o.cpu().numpy()

    call(h1, y1)
    ref = call(h2, y2)
    for v in (22,):
        call(h1, y1, v)
        assert np.array_equal(call(h2, y2), ref), v


def test_class_sums_and_alpha(dev):
    from distributedauc_amd import ops

    rng = np.random.default_rng(5)
    sums = torch.zeros(4, dtype=torch.float64, device=dev)
    ref = np.zeros(4)
    for B in (32, 3000, 100_000):
        h = rng.random(B, dtype=np.float32)
        y = np.where(rng.random(B) < 0.3, 1, -1).astype(np.int8)
        ops.class_sums(T(h, dev), T(y, dev), sums, accumulate=True)
        hd = h.astype(np.float64)
        ref += [hd[y == -1].sum(), (y == -1).sum(), hd[y == 1].sum(), (y == 1).sum()]
    got = sums.cpu().numpy()
    # fp32 partials per 4-element slot folded into fp64: ~1e-7 relative; the reference
    # itself accumulates these sums in fp32 tensors (main.py:166-188)
    assert np.allclose(got, ref, rtol=1e-6, atol=0)
    assert got[1] == ref[1] and got[3] == ref[3]  # counts exact
    alpha = torch.zeros(1, device=dev)
    ops.alpha_from_sums(sums, alpha)
    assert alpha.item() == np.float32(got[0] / got[1] - got[2] / got[3])


def test_label_map_phat_exact(dev):
    from distributedauc_amd import ops

    rng = np.random.default_rng(9)
    for split in (4, 499, 0):
        lab = rng.integers(0, 1000, size=256).astype(np.int64)
        lc = torch.tensor([3.0, 17.0], device=dev)
        gc = torch.tensor([120.0, 901.0], device=dev)
        y8 = torch.empty(256, dtype=torch.int8, device=dev)
        p = torch.zeros(1, device=dev)
        ops.label_map_phat(T(lab, dev), split, y8, lc, gc, p)
        ym = R.label_map(lab, split)
        assert np.array_equal(y8.cpu().numpy(), ym)
        lpos, lneg = 3 + (ym == 1).sum(), 17 + (ym == -1).sum()
        assert lc.cpu().tolist() == [lpos, lneg]
        assert p.cpu().numpy()[0] == R.phat(120.0, 901.0, lpos, lneg)


# ------------------------------------------------------------------ update
def test_pd_update_dense_bitexact(dev):
    from distributedauc_amd import ops

    rng = np.random.default_rng(1)
    for n in (1, 3, 4096, 4097, 1_000_003):
        w, g, w0, avg = (rng.standard_normal(n).astype(np.float32) for _ in range(4))
        tw, tavg = T(w, dev), T(avg, dev)
        ops.pd_update_dense(tw, T(g, dev), T(w0, dev), tavg, lr=0.1 / 3, gamma=2000.0)
        ew, eavg = coracle.pd_update(w, g, w0, 0.1 / 3, 2000.0, avg)
        assert np.array_equal(tw.cpu().numpy(), ew), n
        assert np.array_equal(tavg.cpu().numpy(), eavg), n
        # the torch-CPU restatement (the reference's own op sequence) agrees bit for bit
        assert np.array_equal(R.dppd_sg_flat(w, g, w0, 0.1 / 3, 2000.0), ew)


def test_dppd_sg_golden_generic_path(dev, golden):
    """main.dppd_sg parity through the reference-signature wrapper (per-tensor path)."""
    from distributedauc_amd import main as M

    z = np.load(golden / "dppd_sg.npz")
    torch.manual_seed(5)
    net = torch.nn.Sequential(torch.nn.Linear(40, 30), torch.nn.BatchNorm1d(30), torch.nn.Linear(30, 2)).to(dev)
    names = [n for n, _ in net.named_parameters()]
    off = 0
    model0 = {}
    for (name, p) in net.named_parameters():
        k = p.numel()
        p.data.copy_(T(z["w"][off:off + k].reshape(p.shape), dev))
        p.grad = T(z["g"][off:off + k].reshape(p.shape), dev)
        model0[name] = T(z["w0"][off:off + k].reshape(p.shape), dev)
        off += k
    mk = lambda v: torch.tensor([v], dtype=torch.float32, device=dev)  # noqa: E731
    a, b, al = (mk(v) for v in z["scalars"])
    for t, gv in zip((a, b, al), z["grad3"]):
        t.grad = mk(gv)
    a0, b0, al0 = (mk(v) for v in z["anchor3"])
    M.dppd_sg(net, a, b, al, model0, a0, b0, al0, float(z["lr"]), float(z["gamma"]))
    got = np.concatenate([p.detach().cpu().numpy().reshape(-1) for p in net.parameters()])
    assert np.array_equal(got, z["w_new"])
    assert np.array_equal(np.array([a.item(), b.item(), al.item()], np.float32), z["scalars_new"])
    assert names


def test_pd_update_segments_flat(dev):
    """Flat-buffer update with per-parameter gradient segments of awkward sizes/layouts."""
    from distributedauc_amd.flat import FlatState

    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 5, 3), torch.nn.BatchNorm2d(5), torch.nn.Conv2d(5, 7, 1),
                              torch.nn.Flatten(), torch.nn.Linear(7 * 4 * 4, 2)).to(dev)
    net = net.to(memory_format=torch.channels_last)
    st = FlatState(net)
    st.snapshot_anchor()
    st.anchor[: st.n_params] += 0.01 * torch.randn(st.n_params, device=dev)
    st.reset_average()
    x = torch.randn(4, 3, 6, 6, device=dev).contiguous(memory_format=torch.channels_last)
    net(x).square().sum().backward()
    st.grad3.copy_(torch.tensor([0.3, -0.1, 0.2, 0.0]))
    st.abalpha.copy_(torch.tensor([0.5, 0.25, -0.5]))
    st.anchor3.copy_(torch.tensor([0.4, 0.2, -0.4]))
    before = {n: p.detach().clone() for n, p in net.named_parameters()}
    grads = {n: p.grad.clone() for n, p in net.named_parameters()}
    w0 = {n: torch.as_strided(st.anchor, p.shape, p.stride(), o).clone() for n, p, o, _ in st.entries}
    avg0 = st.avg.clone()
    st.update(0.1, 10.0, "reference")
    for n, p in net.named_parameters():
        e = R.pd_step(before[n].cpu(), grads[n].cpu(), w0[n].cpu(), 0.1, 10.0)
        assert torch.equal(p.detach().cpu(), e), n
    # running average: avg + w_new over every parameter slot
    assert torch.equal(st.avg.cpu(), (avg0 + st.params).cpu())
    ea, eb, eal = R.scalar_update(0.5, 0.25, -0.5, 0.3, -0.1, 0.2, 0.4, 0.2, -0.4, 0.1, 10.0, "reference")
    assert st.abalpha.cpu().numpy().tolist() == [ea, eb, eal]


def test_scalar_update_paper_mode(dev):
    from distributedauc_amd import ops

    sc = torch.tensor([0.5, 0.25, -0.5], device=dev)
    ops.pd_update(sc, sc, None, None, 0, scalars=sc, grad3=torch.tensor([0.3, -0.1, 0.2], device=dev),
                  anchor3=torch.tensor([0.4, 0.2, -0.4], device=dev), lr=0.1, gamma=10.0, mode="paper")
    e = R.scalar_update(0.5, 0.25, -0.5, 0.3, -0.1, 0.2, 0.4, 0.2, -0.4, 0.1, 10.0, "paper")
    assert sc.cpu().numpy().tolist() == list(e)


def test_coda_finalize_and_scale_div(dev):
    from distributedauc_amd import ops

    rng = np.random.default_rng(2)
    for world in (1, 2, 4, 8, 3):
        n = 10_001
        x = rng.standard_normal(n + 5).astype(np.float32)
        x[n + 3:] = [7.0, 29.0]
        tx = T(x, dev)
        gc = torch.tensor([100.0, 400.0], device=dev)
        ops.coda_finalize(tx, n + 3, world, tx[n + 3:n + 5], gc)
        got = tx.cpu().numpy()
        exp = x.copy()
        if world > 1:
            exp[: n + 3] = (torch.from_numpy(x[: n + 3]) / float(world)).numpy()
        assert np.array_equal(got[: n + 3], exp[: n + 3])
        assert got[n + 3:n + 5].tolist() == [0.0, 0.0] and gc.cpu().tolist() == [107.0, 429.0]
    y = rng.standard_normal(777).astype(np.float32)
    ty = T(y, dev)
    ops.scale_div(ty, 15.0)
    assert np.array_equal(ty.cpu().numpy(), (torch.from_numpy(y) / 15).numpy())


# ------------------------------------------------------------------ exact AUC
def _counts_gpu(dev, y, s, world=1, rank=0, variant=0, method="pairs"):
    from distributedauc_amd.auc import ExactAUC

    return ExactAUC(world=world, rank=rank, variant=variant, reduce=False, method=method).counts(T(y, dev),
                                                                                                T(s, dev))


def test_auc_golden(dev, golden):
    from distributedauc_amd.auc import ExactAUC

    z = np.load(golden / "auc_cases.npz")
    for name in z["names"]:
        y, s = z[f"{name}_y"], z[f"{name}_s"]
        W, Tt, P, N, two_u = (int(v) for v in z[f"{name}_counts"])
        for variant in (0, 1, 2, 3, 6):
            c = _counts_gpu(dev, y, s, variant=variant)
            assert (c["wins"], c["ties"], c["P"], c["N"]) == (W, Tt, P, N), (name, variant, c)
            assert 2 * c["wins"] + c["ties"] == two_u
        c = _counts_gpu(dev, y, s, method="sort")
        assert (c["wins"], c["ties"], c["P"], c["N"]) == (W, Tt, P, N), (name, "sort", c)
        auc = ExactAUC.from_counts(c)
        ref = float(z[f"{name}_auc"])
        assert abs(auc - ref) <= 4 * np.spacing(ref), (name, auc, ref)


@pytest.mark.parametrize("n,p,ties", [(1 << 20, 0.01, False), (1 << 20, 0.3, True), (1 << 24, 0.01, False),
                                      (1 << 24, 0.01, True)])
def test_auc_counts_large(dev, n, p, ties):
    """Full-size parity: 2^24 scores at 1 % positives (configs[3]) vs the C oracle, bit-exact."""
    rng = np.random.default_rng(n + int(ties))
    s = rng.random(n, dtype=np.float32)
    if ties:
        s = (np.floor(s * 4096) / 4096).astype(np.float32)
    y = np.where(rng.random(n) < p, 1, -1).astype(np.int8)
    e = coracle.auc_counts(y.astype(np.int64), s)
    for method in ("pairs", "sort"):
        c = _counts_gpu(dev, y, s, method=method)
        assert (c["wins"], c["ties"], c["P"], c["N"]) == (e["wins"], e["ties"], e["P"], e["N"]), method


def test_auc_sharded_sum_is_invariant(dev):
    """Sharding over G ranks (pairs: positive blocks; sort: the larger class, the one streamed
    through the search) sums to the unsharded counts for every G."""
    rng = np.random.default_rng(4)
    n = 300_000
    s = (np.floor(rng.random(n) * 1000) / 1000).astype(np.float32)
    y = np.where(rng.random(n) < 0.05, 1, -1).astype(np.int8)
    full = _counts_gpu(dev, y, s)
    for method in ("pairs", "sort"):
        for G in (2, 3, 4, 8):
            parts = [_counts_gpu(dev, y, s, world=G, rank=r, method=method) for r in range(G)]
            assert sum(c["wins"] for c in parts) == full["wins"]
            assert sum(c["ties"] for c in parts) == full["ties"]


def test_auc_errors_like_sklearn(dev):
    from distributedauc_amd.auc import AUC

    with pytest.raises(ValueError):
        AUC(torch.tensor([1, -1, 1], device=dev), torch.tensor([0.1, float("nan"), 0.3], device=dev))
    with pytest.raises(ValueError):
        AUC(torch.tensor([1, -1, 1], device=dev), torch.tensor([0.1, float("inf"), 0.3], device=dev))
    # three label values: sklearn 1.7.2's roc_curve(pos_label=1) accepts a "multiclass" y_true when
    # pos_label is given and takes every label other than 1 as a negative (0.0 here, like sklearn)
    assert AUC(torch.tensor([1, -1, 0], device=dev), torch.tensor([0.1, 0.2, 0.3], device=dev)) == 0.0
    assert AUC(torch.tensor([1, -1, 0, 1, 2], device=dev), torch.tensor([0.9, 0.1, 0.5, 0.4, 0.3], device=dev)) == (
        pytest.approx(R.auc_sklearn(np.array([1, -1, 0, 1, 2]), np.array([0.9, 0.1, 0.5, 0.4, 0.3], np.float32)),
                      rel=1e-12))
    with pytest.raises(ValueError):  # non-integer float labels: "continuous" for sklearn
        AUC(np.array([1.0, 0.5, 0.0]), np.array([0.1, 0.2, 0.3], np.float32))
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        v = AUC(torch.tensor([1, 1, 1], device=dev), torch.tensor([0.1, 0.2, 0.3], device=dev))
    assert np.isnan(v) and rec
    # {0, 1} labels are binary for sklearn: 0 is the negative class
    assert AUC(np.array([1, 0, 1, 0]), np.array([0.9, 0.1, 0.8, 0.2], np.float32)) == 1.0


def test_split_is_stable(dev):
    from distributedauc_amd import ops

    rng = np.random.default_rng(8)
    n = 123_457
    s = rng.random(n, dtype=np.float32)
    y = np.where(rng.random(n) < 0.2, 1, -1).astype(np.int8)
    pos, neg, stats = ops.split_scores(T(s, dev), T(y, dev))
    P, N, nf, other = stats.cpu().tolist()
    assert (P, N, nf, other) == ((y == 1).sum(), (y != 1).sum(), 0, 0)
    assert np.array_equal(pos[:P].cpu().numpy(), s[y == 1])
    assert np.array_equal(neg[:N].cpu().numpy(), s[y != 1])


@pytest.mark.parametrize("ldtype", [np.int8, np.int32, np.int64])
def test_compact_positives(dev, ldtype):
    """Stable positive compaction (labels read once, positives' scores only): same list as
    s[y == 1], stats = {P, n - P, #non-finite positives, #labels not in {-1, 1}}; ragged sizes
    around the 16-label groups and the 32768-label tile, misaligned label slices, p = 0 / 1,
    growing and shrinking n on one workspace (2^24 + 5: 513 tiles, each summing the counts of
    the tiles before it)."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(31)
    for n, p, off in ((1, 1.0, 0), (15, 0.5, 0), (16, 0.5, 1), (17, 0.3, 0), (16384, 0.01, 0), (32768, 0.01, 0), (32769, 0.0, 0),
                      (32771, 1.0, 3), (300_001, 0.02, 1), (2_000_003, 0.001, 0), (1 << 20, 0.5, 0),
                      ((1 << 24) + 5, 0.3, 0), (40_000, 0.9, 2), (1 << 22, 1.0, 0)):
        sall = rng.standard_normal(n + off).astype(np.float32)
        yall = np.where(rng.random(n + off) < p, 1, -1).astype(ldtype)
        if n > 100:
            yall[rng.random(n + off) < 0.003] = 0  # a negative for roc_curve(pos_label=1), counted as "other"
            sall[rng.integers(0, n + off, 5)] = np.nan
        ts, ty = T(sall, dev)[off:], T(yall, dev)[off:]
        s, y = sall[off:], yall[off:]
        pos, stats = ops.compact_positives(ts, ty)
        P = int((y == 1).sum())
        nf = int((~np.isfinite(s[y == 1])).sum())
        other = int(((y != 1) & (y != -1)).sum())
        assert stats.cpu().tolist() == [P, n - P, nf, other], (n, p, off)
        assert np.array_equal(pos[:P].cpu().numpy(), s[y == 1], equal_nan=True), (n, p, off)


@pytest.mark.parametrize("ldtype", [np.int8, np.int32, np.int64])
def test_auc_eval_counts_one_call(dev, ldtype):
    """dauc_auc_eval_counts (the single-GPU evaluation in one blocking call) vs the C oracle:
    P < N (positives are the table), P > N (split, negatives are the table), P == N, one class
    empty, labels 0 counted as negatives and as "other", a non-finite positive or negative
    reported (and no counts), ragged sizes; and the workspace reused across sizes."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(77)
    cases = [(1, 1.0), (2, 0.5), (1000, 0.0), (1000, 1.0), (4097, 0.5), (300_001, 0.02), (300_001, 0.9),
             (1 << 20, 0.5), (2_000_003, 0.001), (65_536, 0.75)]
    for n, p in cases:
        s = (np.floor(rng.random(n) * 3000) / 3000).astype(np.float32)
        y = np.where(rng.random(n) < p, 1, -1).astype(ldtype)
        if n > 100:
            y[rng.random(n) < 0.002] = 0
        W, Tt, P, N, bad, other = ops.auc_eval_counts(T(s, dev), T(y, dev))
        e = coracle.auc_counts(y.astype(np.int64), s)
        assert (P, N, bad, other) == (e["P"], e["N"], 0, int((y == 0).sum())), (n, p)
        if P and N:
            assert (W, Tt) == (e["wins"], e["ties"]), (n, p)
        else:
            assert (W, Tt) == (0, 0)
    # repeated length, other class sizes (the calls keep no state: each does the same work), both
    # table sides
    n = 300_001
    data = []
    for p in (0.02, 0.03, 0.02, 0.7, 0.02):
        s = rng.random(n, dtype=np.float32)
        data.append((s, np.where(rng.random(n) < p, 1, -1).astype(ldtype)))
    for k in (0, 0, 1, 1, 0, 2, 3, 3, 4, 0):
        s, y = data[k]
        W, Tt, P, N, bad, other = ops.auc_eval_counts(T(s, dev), T(y, dev))
        e = coracle.auc_counts(y.astype(np.int64), s)
        assert (W, Tt, P, N, bad) == (e["wins"], e["ties"], e["P"], e["N"], 0), k
    # the direct count-index build (no sort) and its fallback to the sorted path: tie-heavy and
    # clustered positive tables (a cell of 15+ keys, too many keys per cell) alternate with
    # spread ones of the same length
    n = 200_003
    base = rng.random(n, dtype=np.float32)
    yb = np.where(rng.random(n) < 0.03, 1, -1).astype(ldtype)
    skew = {
        "spread": base,
        "all_equal": np.where(yb == 1, np.float32(0.25), base).astype(np.float32),
        "ten_levels": np.where(yb == 1, np.floor(base * 10) / 10, base).astype(np.float32),
        "cluster": np.where(yb == 1, np.float32(0.5) + base * np.float32(1e-6), base).astype(np.float32),
        "neg_zero": np.where(yb == 1, np.float32(-0.0), np.where(base < 0.5, np.float32(0.0), base)).astype(np.float32),
    }
    for name in ("spread", "all_equal", "all_equal", "spread", "spread", "ten_levels", "cluster", "spread",
                 "neg_zero", "spread"):
        s = skew[name]
        W, Tt, P, N, bad, other = ops.auc_eval_counts(T(s, dev), T(yb, dev))
        e = coracle.auc_counts(yb.astype(np.int64), s)
        assert (W, Tt, P, N, bad) == (e["wins"], e["ties"], e["P"], e["N"], 0), name
    for where in ("pos", "neg"):
        for p in (0.01, 0.99):  # both table sides
            n = 100_003
            s = rng.random(n, dtype=np.float32)
            y = np.where(rng.random(n) < p, 1, -1).astype(ldtype)
            j = int(np.flatnonzero(y == (1 if where == "pos" else -1))[3])
            s[j] = np.inf if where == "pos" else np.nan
            W, Tt, P, N, bad, other = ops.auc_eval_counts(T(s, dev), T(y, dev))
            assert bad >= 1, (where, p)


@pytest.mark.parametrize("ldtype", [np.int8, np.int32, np.int64])
def test_auc_eval_counts_wide_tiles(dev, ldtype):
    """From 2^25 labels the one-pass compaction takes 131072-label tiles whose label loads go out
    in straight-line batches when the tile is wholly in range and aligned (DAUC_COMPACT_BATCH);
    a ragged last tile and a misaligned label slice take the per-group bounds-checked path. Both,
    for every label width, against the C oracle (2^25 + 7 labels, 0.1 % positives)."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(2025)
    n = (1 << 25) + 7
    for off in (0, 1):
        sall = (np.floor(rng.random(n + off) * 50_000) / 50_000).astype(np.float32)
        yall = np.where(rng.random(n + off) < 0.001, 1, -1).astype(ldtype)
        yall[rng.random(n + off) < 1e-5] = 0  # counted as a negative and as "other"
        s, y = sall[off:], yall[off:]
        W, Tt, P, N, bad, other = ops.auc_eval_counts(T(sall, dev)[off:], T(yall, dev)[off:])
        e = coracle.auc_counts(y.astype(np.int64), s)
        assert (W, Tt, P, N, bad, other) == (e["wins"], e["ties"], e["P"], e["N"], 0, int((y == 0).sum())), off


def test_auc_eval_counts_stale_workspace(dev):
    """The evaluation re-initialises every byte of state it reads (one memset of the workspace
    header per call): a workspace overwritten with garbage between calls (as a freed-and-
    reallocated buffer would be) still gives the C oracle's counts, and nothing is written out of
    bounds."""
    from distributedauc_amd import _lib, ops

    rng = np.random.default_rng(12)
    n = 300_001
    s = rng.random(n, dtype=np.float32)
    y = np.where(rng.random(n) < 0.02, 1, -1).astype(np.int8)
    e = coracle.auc_counts(y.astype(np.int64), s)
    st, sy = T(s, dev), T(y, dev)
    want = (e["wins"], e["ties"], e["P"], e["N"], 0, 0)
    assert ops.auc_eval_counts(st, sy) == want
    ws = ops.workspaces.get(dev, "auc_eval", _lib.load().dauc_auc_eval_workspace_size(n),
                            torch.cuda.current_stream(dev).cuda_stream)
    for fill in (0xAB, 0x00, 0xFF):
        assert ops.auc_eval_counts(st, sy) == want
        ws.fill_(fill)
        assert ops.auc_eval_counts(st, sy) == want, fill
        assert ops.auc_eval_counts(st, sy) == want, fill
    torch.cuda.synchronize()


def test_auc_eval_counts_part(dev):
    """dauc_auc_eval_counts_part (the sharded evaluation's per-rank call): for G = 1, 2, 3, 8 the
    parts' (W, T) sum to the C oracle's on both table sides (P < N: score ranges; P > N: positive
    ranges), including G larger than a tiny n (empty parts); the device part_counts equal the host
    ones; P, N and the global checks are the same on every part; a non-finite negative shows up
    in exactly the part whose range holds it."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(91)
    for n, p in ((300_001, 0.02), (300_001, 0.8), (5, 0.4), (2_000_003, 0.001), (300_001, 0.03)):
        s = (np.floor(rng.random(n) * 2000) / 2000).astype(np.float32)
        y = np.where(rng.random(n) < p, 1, -1).astype(np.int8)
        e = coracle.auc_counts(y.astype(np.int64), s)
        for G in (1, 2, 3, 8):
            W = Tt = 0
            for r in range(G):
                pc = torch.full((3,), -7, dtype=torch.int64, device=dev)
                o = ops.auc_eval_counts_part(T(s, dev), T(y, dev), r, G, pc)
                assert o[2:6] == (e["P"], e["N"], 0, 0) and o[6] == 0, (n, p, G, r, o)
                if e["P"] and e["N"]:
                    assert pc.cpu().tolist() == [o[0], o[1], 0], (n, p, G, r)
                W += o[0]
                Tt += o[1]
            if e["P"] and e["N"]:
                assert (W, Tt) == (e["wins"], e["ties"]), (n, p, G)
    n = 100_003
    s = rng.random(n, dtype=np.float32)
    y = np.where(rng.random(n) < 0.05, 1, -1).astype(np.int8)
    j = int(np.flatnonzero(y == -1)[-2])  # in the last part's range
    s[j] = np.nan
    pc = torch.zeros(3, dtype=torch.int64, device=dev)
    seen = [ops.auc_eval_counts_part(T(s, dev), T(y, dev), r, 4, pc)[6] for r in range(4)]
    assert seen == [0, 0, 0, 1], seen


def test_auc_eval_enqueue_records(dev):
    """dauc_auc_eval_enqueue (the sharded evaluation's per-rank part, no host synchronisation): for
    G = 1, 2, 3, 8 the parts' W, T sum to the C oracle's; P, the non-finite and label counts are
    the same in every part's record; verdict 1 where the count index holds the table, 0 for an
    empty part (G > n), and 2 on EVERY part for tables it cannot hold (more positives than
    n / 2 + 1, a tie-heavy or clustered table) -- the blocking part then gives the oracle's
    integers; a NaN negative is counted in exactly the part that queries it."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(93)
    base = rng.random(300_001, dtype=np.float32)
    cases = []
    for p in (0.02, 0.001, 0.6):
        cases.append(("spread", p, base, np.where(rng.random(base.size) < p, 1, -1).astype(np.int8)))
    yb = np.where(rng.random(base.size) < 0.03, 1, -1).astype(np.int8)
    cases.append(("all_equal", 0.03, np.where(yb == 1, np.float32(0.25), base).astype(np.float32), yb))
    cases.append(("cluster", 0.03, np.where(yb == 1, np.float32(0.5) + base * np.float32(1e-6), base).astype(np.float32), yb))
    cases.append(("tiny", 0.4, base[:5].copy(), np.array([1, -1, -1, 1, -1], np.int8)))
    for name, p, s, y in cases:
        e = coracle.auc_counts(y.astype(np.int64), s)
        for G in (1, 2, 3, 8):
            recs = []
            for r in range(G):
                out = torch.full((8,), -7, dtype=torch.int64, device=dev)
                ops.auc_eval_enqueue(T(s, dev), T(y, dev), r, G, out=out)
                recs.append(out.cpu().tolist())
            assert {(v[3], v[4], v[5], v[6]) for v in recs} == {(e["P"], 0, 0, 0)}, (name, G, recs)
            verdicts = {v[7] for v in recs} - {0}
            assert len(verdicts) == 1, (name, G, recs)
            n = s.size
            if G > n:
                assert any(v[7] == 0 and v[0] == v[1] == 0 for v in recs)
            fits = name in ("spread", "tiny") and e["P"] <= n // 2 + 1
            if name != "cluster":  # a clustered table may or may not overflow a cell: either is exact
                assert verdicts == ({1} if fits else {2}), (name, G, verdicts)
            if verdicts == {1}:
                assert (sum(v[0] for v in recs), sum(v[1] for v in recs)) == (e["wins"], e["ties"]), (name, G)
                assert sum(v[2] for v in recs) == 0
            else:
                W = Tt = 0
                for r in range(G):
                    pc = torch.zeros(3, dtype=torch.int64, device=dev)
                    o = ops.auc_eval_counts_part(T(s, dev), T(y, dev), r, G, pc)
                    W, Tt = W + o[0], Tt + o[1]
                assert (W, Tt) == (e["wins"], e["ties"]), (name, G)
    s = rng.random(100_003, dtype=np.float32)
    y = np.where(rng.random(s.size) < 0.05, 1, -1).astype(np.int8)
    s[int(np.flatnonzero(y == -1)[-2])] = np.nan  # in the last part's range
    seen = [ops.auc_eval_enqueue(T(s, dev), T(y, dev), r, 4)[2].item() for r in range(4)]
    assert seen == [0, 0, 0, 1], seen


@pytest.mark.parametrize("ldtype", [np.int8, np.int32, np.int64])
def test_auc_eval_bucketed_ranges(dev, ldtype):
    """The count-index evaluation against the C oracle on distributions that once stressed round
    3's range-bucketed count (removed; the cases stay for the count index and its cell map): few
    positives and ~220 k positives (near the index's capacity); every query in one narrow
    interval; queries in top buckets with no positive at all (their cell is the next used bucket's
    first); queries below / above every positive; a misaligned score slice and misaligned labels;
    parts with ragged bounds (G = 3, 7)."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(404)
    n = 1_000_003
    u = rng.random(n, dtype=np.float32)
    cases = {
        "one_range": (u, np.where(rng.random(n) < 0.002, 1, -1)),
        "max_ranges": (u, np.where(rng.random(n) < 0.21, 1, -1)),
        "queries_one_range": None,
        "apart": None,
        "outside": None,
    }
    y = np.where(rng.random(n) < 0.05, 1, -1)
    s = np.where(y == 1, u, np.float32(0.6) + u * np.float32(1e-4)).astype(np.float32)
    cases["queries_one_range"] = (s, y)
    s = np.where(y == 1, np.float32(0.5) + u * np.float32(0.5), u * np.float32(1e-3)).astype(np.float32)
    cases["apart"] = (s, y)  # negatives in top buckets with no positive
    s = np.where(y == 1, np.float32(0.4) + u * np.float32(0.2), np.where(u < 0.5, -u, np.float32(1) + u))
    cases["outside"] = (s.astype(np.float32), y)
    for name, (s, y) in cases.items():
        y = y.astype(ldtype)
        e = coracle.auc_counts(y.astype(np.int64), s)
        W, Tt, P, N, bad, other = ops.auc_eval_counts(T(s, dev), T(y, dev))
        assert (W, Tt, P, N, bad, other) == (e["wins"], e["ties"], e["P"], e["N"], 0, 0), name
        for G in (3, 7):
            Wp = Tp = 0
            for r in range(G):
                out = torch.zeros(8, dtype=torch.int64, device=dev)
                ops.auc_eval_enqueue(T(s, dev), T(y, dev), r, G, out=out)
                v = out.cpu().tolist()
                assert v[7] in (0, 1), (name, G, r, v)
                Wp, Tp = Wp + v[0], Tp + v[1]
            assert (Wp, Tp) == (e["wins"], e["ties"]), (name, G)
    # misaligned slices: scores off by 1 element (4 B: the split's scalar path), labels by 1
    s, y = cases["max_ranges"][0], cases["max_ranges"][1].astype(ldtype)
    for so, yo in ((1, 0), (0, 1), (3, 2)):
        sall = np.concatenate([np.zeros(so, np.float32), s])
        yall = np.concatenate([np.zeros(yo, ldtype), y])
        e = coracle.auc_counts(y.astype(np.int64), s)
        W, Tt, P, N, bad, other = ops.auc_eval_counts(T(sall, dev)[so:], T(yall, dev)[yo:])
        assert (W, Tt, P, N, bad) == (e["wins"], e["ties"], e["P"], e["N"], 0), (so, yo)


def test_auc_one_class_rejects_nonfinite(dev):
    """with one class empty, a non-finite score must still raise like sklearn
    (roc_curve checks finiteness before its one-class warning), one GPU and sharded."""
    from distributedauc_amd.auc import ExactAUC

    n = 50_003
    rng = np.random.default_rng(17)
    for fill in (-1, 1):
        s = rng.random(n, dtype=np.float32)
        y = np.full(n, fill, np.int8)
        s[n // 3] = np.nan
        with pytest.raises(ValueError):
            ExactAUC(method="sort")(T(y, dev), T(s, dev))
        hits = 0
        for r in range(3):
            try:
                ExactAUC(world=3, rank=r, reduce=False, method="sort", shard_min=0).counts(T(y, dev), T(s, dev))
            except ValueError:
                hits += 1
        # a non-finite negative is seen by the part that queries it; a non-finite positive by the
        # compaction, i.e. by every part that compacts it
        assert hits >= 1, fill


def _two_step(dev, s, y, G):
    """The two-step sharded evaluation on one device: every part's slot compacted, the slots
    concatenated as an all-gather would, then every part's query; returns the G records."""
    from distributedauc_amd import ops

    n = s.size
    nb = ops.auc_slot_bytes(n, G)
    slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
    ts, ty = T(s, dev), T(y, dev)
    for r in range(G):
        mine = torch.empty(nb, dtype=torch.uint8, device=dev)
        ops.auc_eval_compact_part(ts, ty, r, G, mine)
        slots[r * nb:(r + 1) * nb].copy_(mine)
    recs = []
    for r in range(G):
        # rank r's own step 1 just before its step 2 (the simulated ranks share one workspace, and
        # step 2 consumes the build state step 1 prepares there)
        ops.auc_eval_compact_part(ts, ty, r, G, mine)
        recs.append(ops.auc_eval_query_part(ts, ty, r, G, slots).cpu().tolist())
    return recs


@pytest.mark.parametrize("ldtype", [np.int8, np.int32, np.int64])
def test_auc_eval_two_step_parts(dev, ldtype):
    """dauc_auc_eval_compact_part + dauc_auc_eval_query_part (each rank compacts
    only its slice; the gathered slots are the table) against the C oracle for G = 1, 2, 3, 8:
    the parts' (W, T) sum to the oracle's, every record carries the same P and label counts;
    an unshuffled test set whose positives crowd one slice overflows that slot and every part
    reports verdict 2 (then the blocking sorted path gives the oracle's integers); a tie-heavy
    table gives verdict 2; a NaN negative is counted in exactly the part that queries it; a NaN
    positive is in every record."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(606)
    n = 300_007
    s = (np.floor(rng.random(n) * 5000) / 5000).astype(np.float32)
    for p in (0.02, 0.2, 0.0005):
        y = np.where(rng.random(n) < p, 1, -1).astype(ldtype)
        y[rng.random(n) < 0.001] = 0
        e = coracle.auc_counts(y.astype(np.int64), s)
        for G in (1, 2, 3, 8):
            recs = _two_step(dev, s, y, G)
            assert {(v[3], v[4], v[5], v[6]) for v in recs} == {(e["P"], 0, 0, int((y == 0).sum()))}, (p, G)
            verdicts = {v[7] for v in recs}
            # 5000 score levels: at p = 0.2 every level holds ~12 positives, so cells of 15+ keys
            # make the index refuse the table (verdict 2 on every part: the blocking sorted path)
            assert verdicts == ({2} if p == 0.2 else {1}), (p, G, recs)
            if verdicts == {1}:
                assert (sum(v[0] for v in recs), sum(v[1] for v in recs)) == (e["wins"], e["ties"]), (p, G)
            else:
                W = Tt = 0
                for r in range(G):
                    o = ops.auc_eval_counts_part(T(s, dev), T(y, dev), r, G,
                                                 torch.zeros(3, dtype=torch.int64, device=dev))
                    W, Tt = W + o[0], Tt + o[1]
                assert (W, Tt) == (e["wins"], e["ties"]), (p, G)
    # unshuffled: every positive in the first slice
    y = np.where(np.arange(n) < 30_000, 1, -1).astype(ldtype)  # slice 0 holds 30000 > its slot (23502)
    e = coracle.auc_counts(y.astype(np.int64), s)
    recs = _two_step(dev, s, y, 8)
    assert {v[7] for v in recs} == {2} and {v[3] for v in recs} == {e["P"]}, recs
    W = Tt = 0
    for r in range(8):
        o = ops.auc_eval_counts_part(T(s, dev), T(y, dev), r, 8, torch.zeros(3, dtype=torch.int64, device=dev))
        W, Tt = W + o[0], Tt + o[1]
    assert (W, Tt) == (e["wins"], e["ties"])
    # tie-heavy positives: the index refuses the table
    y = np.where(rng.random(n) < 0.03, 1, -1).astype(ldtype)
    s2 = np.where(y == 1, np.float32(0.25), s).astype(np.float32)
    assert {v[7] for v in _two_step(dev, s2, y, 3)} == {2}
    # a NaN negative in the last slice: counted by the part that queries it (part r queries slice
    # r + 1); a NaN positive in every record
    s3 = s.copy()
    s3[int(np.flatnonzero(y == -1)[-2])] = np.nan
    assert [v[2] for v in _two_step(dev, s3, y, 4)] == [0, 0, 1, 0]
    s4 = s.copy()
    s4[int(np.flatnonzero(y == 1)[0])] = np.nan
    assert {v[5] for v in _two_step(dev, s4, y, 4)} == {1}


def test_auc_eval_records_counted_in_place(dev):
    """The enqueued forms count straight into the caller's part_out (no copy from the workspace):
    a record holding garbage, or the previous call's counts, comes back exactly the fresh record
    (the enqueue's memset, the query part's gather zero it first); two parts' records side by side
    in one buffer do not disturb each other."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(31)
    n = 200_003
    s = rng.random(n, dtype=np.float32)
    y = np.where(rng.random(n) < 0.01, 1, -1).astype(np.int8)
    e = coracle.auc_counts(y.astype(np.int64), s)
    ts, ty = T(s, dev), T(y, dev)
    G = 2
    nb = ops.auc_slot_bytes(n, G)
    slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
    for r in range(G):
        ops.auc_eval_compact_part(ts, ty, r, G, slots[r * nb:(r + 1) * nb])
    recs = torch.full((8 * G,), -0x0123456789ABCDEF, dtype=torch.int64, device=dev)
    mine = torch.empty(nb, dtype=torch.uint8, device=dev)
    for rep in range(2):
        for r in range(G):
            ops.auc_eval_compact_part(ts, ty, r, G, mine)  # rank r's step 1 (the build state step 2 consumes)
            ops.auc_eval_query_part(ts, ty, r, G, slots, out=recs[8 * r:8 * (r + 1)])
        v = recs.view(G, 8).cpu().tolist()
        assert (sum(x[0] for x in v), sum(x[1] for x in v)) == (e["wins"], e["ties"]), rep
        assert all(x[3] == e["P"] and x[4] == 0 and x[7] == 1 for x in v), (rep, v)
        recs.fill_(-1)
        for r in range(G):
            ops.auc_eval_enqueue(ts, ty, r, G, out=recs[8 * r:8 * (r + 1)])
        w = recs.view(G, 8).cpu().tolist()
        # the two forms split the queries differently (the enqueue's part r counts [rn/G, (r+1)n/G),
        # the query part's the next slice): same sums, same per-record counts otherwise
        assert (sum(x[0] for x in w), sum(x[1] for x in w)) == (e["wins"], e["ties"]), rep
        assert [x[2:] for x in w] == [x[2:] for x in v], (rep, w, v)


@pytest.mark.parametrize("n,G", [(300_007, 3), ((1 << 25) + 4097, 1)])
def test_auc_eval_slot_layout(dev, n, G):
    """The slot dauc_auc_eval_compact_part writes is the CPU stand-in's (tests/cpu_kernels.py):
    the header, the top-bucket histogram of the slice's positives (count_index.h keys: -0 on +0,
    NaN and +-inf included) and the positives themselves (as a multiset: the compaction keeps no
    order). 2^25 labels in one slice take the wide compaction tiles."""
    import cpu_kernels
    from distributedauc_amd import ops

    rng = np.random.default_rng(77)
    s = (rng.standard_normal(n) * 3).astype(np.float32)
    y = np.where(rng.random(n) < 0.002, 1, -1).astype(np.int8)
    pos_idx = np.flatnonzero(y == 1)
    s[pos_idx[:4]] = np.array([0.0, -0.0, np.inf, np.nan], np.float32)
    y[5] = 0
    nb = ops.auc_slot_bytes(n, G)
    assert nb == cpu_kernels.auc_slot_bytes(n, G)
    ts, ty = T(s, dev), T(y, dev)
    for r in range(G):
        got = torch.full((nb,), 0xAB, dtype=torch.uint8, device=dev)
        ops.auc_eval_compact_part(ts, ty, r, G, got)
        want = cpu_kernels.auc_eval_compact_part(torch.from_numpy(s), torch.from_numpy(y), r, G,
                                                 torch.zeros(nb, dtype=torch.uint8))
        g, w = got.cpu().numpy(), want.numpy()
        assert np.array_equal(g[:40], w[:40]), r  # P, 0, non-finite, other, n
        assert np.array_equal(g[256:8448], w[256:8448]), r
        k = int(w[:8].view(np.int64)[0])
        gp, wp = g[8448:8448 + 4 * k].view(np.uint32), w[8448:8448 + 4 * k].view(np.uint32)
        assert np.array_equal(np.sort(gp), np.sort(wp)), r


def test_auc_sort_rejects_nonfinite_negatives(dev):
    """The sort method never materialises the negatives: the query kernel's finiteness count
    must still reject a NaN / inf negative (sklearn _ranking.py:868-869), sharded or not."""
    from distributedauc_amd.auc import ExactAUC

    rng = np.random.default_rng(5)
    n = 200_003
    for bad in (np.nan, np.inf, -np.inf):
        s = rng.random(n, dtype=np.float32)
        y = np.where(rng.random(n) < 0.01, 1, -1).astype(np.int8)
        j = int(np.flatnonzero(y == -1)[-7])
        s[j] = bad
        with pytest.raises(ValueError):
            ExactAUC(method="sort")(T(y, dev), T(s, dev))
        # two shards: only the rank whose slice holds the bad score sees it before the reduce
        hits = 0
        for r in range(2):
            try:
                ExactAUC(world=2, rank=r, reduce=False, method="sort").counts(T(y, dev), T(s, dev))
            except ValueError:
                hits += 1
        assert hits == 1


def test_auc_counts_extreme_configs4(dev):
    """BASELINE configs[4] at full size: 2^27 fp32 scores at 0.1 % positives, drawn by the
    bench's own generator (loader.synthetic_scores), both exact methods, bit-exact vs the C
    oracle's O(n log n) integer counts; sort-method shards over 8 ranks sum to the same."""
    from distributedauc_amd.auc import ExactAUC
    from distributedauc_amd.loader import synthetic_scores

    ts, ty = synthetic_scores(1 << 27, 0.001, dev)
    e = coracle.auc_counts(ty.cpu().numpy().astype(np.int64), ts.cpu().numpy())
    ref = (e["wins"], e["ties"], e["P"], e["N"])
    for method in ("sort", "pairs"):
        c = ExactAUC(method=method).counts(ty, ts)
        assert (c["wins"], c["ties"], c["P"], c["N"]) == ref, method
    parts = [ExactAUC(world=8, rank=r, reduce=False).counts(ty, ts) for r in range(8)]
    assert (sum(c["wins"] for c in parts), sum(c["ties"] for c in parts)) == ref[:2]


def test_pair_count_edge_sizes(dev):
    from distributedauc_amd import ops

    rng = np.random.default_rng(6)
    for P, N in ((1, 1), (1, 5000), (3000, 1), (2049, 2047), (4097, 9001), (0, 10), (10, 0)):
        pos = (np.floor(rng.random(P) * 64) / 64).astype(np.float32)
        neg = (np.floor(rng.random(N) * 64) / 64).astype(np.float32)
        for variant in range(12):
            wt = torch.zeros(2, dtype=torch.int64, device=dev)
            ops.pair_count(T(pos, dev), T(neg, dev), wt, variant=variant)
            assert tuple(wt.cpu().tolist()) == coracle.pair_count_bruteforce(pos, neg), (P, N, variant)
    # misaligned negative base pointer (sharded slices)
    pos = rng.random(777, dtype=np.float32)
    negall = rng.random(10_001, dtype=np.float32)
    tn = T(negall, dev)
    wt = torch.zeros(2, dtype=torch.int64, device=dev)
    ops.pair_count(T(pos, dev), tn[1:], wt)
    assert tuple(wt.cpu().tolist()) == coracle.pair_count_bruteforce(pos, negall[1:])




@pytest.mark.parametrize("variant", [0, 4, 8, 1])
def test_pair_count_packed_fallback_values(dev, variant):
    """Mode 0 (packed fp32 difference + clamp) must equal exact compares for every value class.

    Tiles are 2048 negatives and blocks 256*RP positives: the unsafe values (+-inf, subnormals,
    |v| < 2^-103) are placed in some tiles / blocks only, so both the packed loop and the
    per-tile compare fallback run inside one launch. Bit-exact vs the C brute-force oracle."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(100 + variant)
    safe = np.array([0.0, -0.0, 1.0, -1.0, 2.0 ** -103, -(2.0 ** -103), 2.0 ** -102, 3.0e38, -3.0e38,
                     1.1754944e-38 * 4096, 0.5, 0.25], np.float32)
    unsafe = np.array([np.inf, -np.inf, 1e-45, -1e-45, 1.1754944e-38, 2.0 ** -104, 1e-40], np.float32)
    for P, N, frac_bad in ((3000, 9000, 0.0), (3000, 9000, 0.002), (5000, 20_000, 0.0005), (17, 5000, 0.01)):
        pool = np.concatenate([safe, rng.random(64, dtype=np.float32), -rng.random(64, dtype=np.float32)])
        pos = rng.choice(pool, P).astype(np.float32)
        neg = rng.choice(pool, N).astype(np.float32)
        # unsafe values only in the second half of the negatives and the last positives
        if frac_bad:
            k = max(1, int(N * frac_bad))
            neg[N // 2 + rng.integers(0, N - N // 2, k)] = rng.choice(unsafe, k)
            pos[-max(1, int(P * frac_bad)):] = rng.choice(unsafe, max(1, int(P * frac_bad)))
        wt = torch.zeros(2, dtype=torch.int64, device=dev)
        ops.pair_count(T(pos, dev), T(neg, dev), wt, variant=variant)
        assert tuple(wt.cpu().tolist()) == coracle.pair_count_bruteforce(pos, neg), (P, N, frac_bad)
    # tiny-difference neighbours: consecutive floats just above the 2^-103 bound and near 1.0
    base = np.array([2.0 ** -103, 1.0, 1e-20], np.float32)
    vals = np.concatenate([np.nextafter(base, np.float32(np.inf)), base])
    pos = np.tile(vals, 300).astype(np.float32)
    neg = np.tile(vals[::-1], 700).astype(np.float32)
    wt = torch.zeros(2, dtype=torch.int64, device=dev)
    ops.pair_count(T(pos, dev), T(neg, dev), wt, variant=variant)
    assert tuple(wt.cpu().tolist()) == coracle.pair_count_bruteforce(pos, neg)

def test_radix_sort_keys(dev):
    """The LSD radix sort orders keys exactly like the floats (with -0 == +0)."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(12)
    for n in (1, 7, 4096, 4097, 300_001):
        v = rng.standard_normal(n).astype(np.float32) * rng.choice([1e-40, 1.0, 1e30], n).astype(np.float32)
        v[rng.random(n) < 0.05] = 0.0
        v[rng.random(n) < 0.05] = -0.0
        k = ops.sort_keys(T(v, dev)).cpu().numpy().view(np.uint32)
        assert np.all(k[1:] >= k[:-1]), n
        u = np.sort(v.copy()).view(np.uint32)
        u = np.where(np.sort(v) == 0, np.uint32(0x80000000), np.where(u >> 31, ~u, u | np.uint32(0x80000000)))
        assert np.array_equal(k, u.astype(np.uint32)), n


@pytest.mark.parametrize("P,N", [(1, 1), (5, 100_000), (100_000, 5), (50_000, 50_000), (3, 4096), (4096, 4097)])
def test_sorted_counts_match_pair_count(dev, P, N):
    from distributedauc_amd import ops

    rng = np.random.default_rng(P * 7 + N)
    pos = (np.floor(rng.random(P) * 97) / 97 - 0.5).astype(np.float32)
    neg = (np.floor(rng.random(N) * 97) / 97 - 0.5).astype(np.float32)
    neg[rng.random(N) < 0.1] = -0.0
    a = torch.zeros(2, dtype=torch.int64, device=dev)
    b = torch.zeros(2, dtype=torch.int64, device=dev)
    ops.pair_count(T(pos, dev), T(neg, dev), a)
    ops.auc_counts_sorted(T(pos, dev), T(neg, dev), b)
    assert a.tolist() == b.tolist()
    if P * N <= 10_000_000:
        assert tuple(a.tolist()) == coracle.pair_count_bruteforce(pos, neg)


@pytest.mark.parametrize("M,L,table_pos", [(10_000, 300_000, True), (20_000, 50_000, True), (60_000, 70_000, False),
                                            (100_000, 2_000_000, True), (250_000, 260_000, False),
                                            (400_000, 1_000_000, True), (600_000, 700_000, True),
                                            (700_000, 600_000, False), (1_100_000, 1_300_000, True)])
def test_sorted_counts_bucket_sizes(dev, M, L, table_pos):
    """The search tree holds every k-th key of the sorted smaller class (<= 32767 splitters, so
    these sizes give k = 1, 2, 4, 8, 16, 32 (one bucket load) and 64 (k > 32: binary search in
    global memory)). Every k, and both table sides, vs the pair-count
    kernel on tie-heavy scores (ties at splitter boundaries included), bit-exact."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(M + L)
    P, N = (M, L) if table_pos else (L, M)
    pos = (np.floor(rng.random(P) * 5003) / 5003 - 0.3).astype(np.float32)
    neg = (np.floor(rng.random(N) * 5003) / 5003 - 0.5).astype(np.float32)
    neg[rng.random(N) < 0.05] = -0.0
    pos[rng.random(P) < 0.05] = 0.0
    a = torch.zeros(2, dtype=torch.int64, device=dev)
    b = torch.zeros(2, dtype=torch.int64, device=dev)
    ops.pair_count(T(pos, dev), T(neg, dev), a)
    ops.auc_counts_sorted(T(pos, dev), T(neg, dev), b)
    assert a.tolist() == b.tolist()
    if M <= 20_000 and L <= 300_000:
        assert tuple(b.tolist()) == coracle.pair_count_bruteforce(pos, neg)


@pytest.mark.parametrize("ldtype", [np.int8, np.int32, np.int64])
@pytest.mark.parametrize("n,p,begin,trim", [(1000, 0.3, 0, 0), (300_001, 0.02, 3, 5), (2_000_003, 0.01, 1, 2),
                                            (150_000, 0.2, 0, 1)])
def test_sorted_counts_labeled(dev, ldtype, n, p, begin, trim):
    """Negatives read in place from [begin, end) of the full arrays (labels != 1, including
    labels outside {-1, 1}) vs the pair-count kernel over the same negatives; unaligned ranges,
    every label dtype, ties and +-0, bit-exact."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(n + begin)
    s = (np.floor(rng.random(n) * 3001) / 3001 - 0.5).astype(np.float32)
    s[rng.random(n) < 0.03] = -0.0
    y = np.where(rng.random(n) < p, 1, -1).astype(ldtype)
    y[rng.random(n) < 0.01] = 0  # not +1: a negative for roc_curve(pos_label=1)
    end = n - trim
    pos = s[y == 1]
    neg = s[begin:end][y[begin:end] != 1]
    a = torch.zeros(2, dtype=torch.int64, device=dev)
    b = torch.zeros(2, dtype=torch.int64, device=dev)
    ops.pair_count(T(pos, dev), T(neg, dev), a)
    ops.auc_counts_sorted_labeled(T(pos, dev), T(s, dev), T(y, dev), begin, end, b)
    assert a.tolist() == b.tolist()


@pytest.mark.parametrize("zdtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B", [1, 256, 5000])
def test_surrogate_logits_fused_softmax(dev, zdtype, B):
    """§8f row 2: loss/grads from logits vs fp64 closed form; dz vs torch autograd through softmax."""
    from distributedauc_amd import ops
    from distributedauc_amd.surrogate import auc_surrogate_logits

    rng = np.random.default_rng(B)
    z = torch.from_numpy(rng.normal(0, 2, (B, 2)).astype(np.float32)).to(dev).to(zdtype)
    y = np.where(rng.random(B) < 0.3, 1, -1).astype(np.int8)
    y[rng.random(B) < 0.05] = 0
    ab = torch.tensor([0.2, -0.1, 0.05], device=dev)
    p = torch.tensor([0.3], device=dev)
    out64 = torch.zeros(6, dtype=torch.float64, device=dev)
    h_out = torch.empty(B, device=dev)
    dz = torch.empty_like(z)
    ops.surrogate_logits_fwdbwd(z, T(y, dev), ab, p, dz=dz, h_out=h_out, out64=out64)
    zf = z.float().cpu().numpy().astype(np.float64)
    h64 = 1.0 / (1.0 + np.exp(zf[:, 0] - zf[:, 1]))
    assert np.allclose(h_out.cpu().numpy(), h64, rtol=2e-6, atol=1e-7)
    F, dh64, da, db, dal = R.surrogate_closed_form(h64.astype(np.float32), y.astype(np.int64), 0.2, -0.1, 0.05,
                                                   np.float32(0.3))
    sc = _scales(h64, y, 0.2, -0.1, 0.05, float(np.float32(0.3)))
    assert np.all(np.abs(out64.cpu().numpy()[:4] - [F, da, db, dal]) <= 1e-5 * sc + 1e-12)
    # autograd of the reference expression through torch's softmax, fp32
    zt = z.float().detach().clone().requires_grad_(True)
    hh = torch.softmax(zt, dim=1)[:, 1]
    Fr = R.surrogate_loss(hh, T(y.astype(np.int64), dev), ab[0], ab[1], ab[2], p[0])
    Fr.backward()
    ref = zt.grad.cpu().numpy()
    got = dz.float().cpu().numpy()
    tol = 1e-5 if zdtype == torch.float32 else 8e-3  # bf16 output rounding (8-bit mantissa)
    scale = np.abs(ref).max() + 1e-12
    assert np.all(np.abs(got - ref) <= tol * np.maximum(np.abs(ref), 1e-3 * scale) + 1e-9), zdtype
    # through autograd: loss.backward() delivers dz to the producer of z
    zz = z.detach().clone().requires_grad_(True)
    g3 = torch.zeros(3, device=dev)
    loss = auc_surrogate_logits(zz, T(y, dev), ab, p, g3)
    loss.backward()
    assert torch.equal(zz.grad, dz)
    assert abs(loss.item() - F) <= 1e-5 * sc[0] + 1e-7


def test_class_sums_logits(dev):
    from distributedauc_amd import ops

    rng = np.random.default_rng(3)
    z = torch.from_numpy(rng.normal(0, 1, (3000, 2)).astype(np.float32)).to(dev)
    y = np.where(rng.random(3000) < 0.3, 1, -1).astype(np.int8)
    s4 = torch.zeros(4, dtype=torch.float64, device=dev)
    ops.class_sums_logits(z, T(y, dev), s4, accumulate=False)
    h = torch.softmax(z.double(), 1)[:, 1].cpu().numpy()
    ref = [h[y == -1].sum(), (y == -1).sum(), h[y == 1].sum(), (y == 1).sum()]
    assert np.allclose(s4.cpu().numpy(), ref, rtol=1e-6)
