"""Tensor-level wrappers over the libdauc.so C ABI.

Every function takes torch tensors that live on the GPU, validates shapes,
dtypes and devices on the host (so a kernel never sees an operand its grid does
not expect), and enqueues the HIP kernel on torch's current stream for that
device. Nothing here synchronises or allocates on the steady-state path except
cached, zero-initialised workspaces. CPU tensors are rejected: there is no CPU
fallback in the product path.
"""
from __future__ import annotations

import ctypes
import threading

import torch

from . import _lib
from ._lib import GradSeg, check

_LABEL_CODES = {torch.int8: _lib.LABEL_I8, torch.int32: _lib.LABEL_I32, torch.int64: _lib.LABEL_I64}
_MODES = {"reference": _lib.MODE_REFERENCE, "paper": _lib.MODE_PAPER}


def _require_gpu(t: torch.Tensor, name: str) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor, got {type(t).__name__}")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{name}: distributedauc_amd runs its hot path on the MI355X only (HIP kernels in "
            f"libdauc.so); got a tensor on {t.device}. There is no CPU fallback."
        )


def _require(t: torch.Tensor, name: str, dtype: torch.dtype, device=None) -> None:
    _require_gpu(t, name)
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")


def _ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _stream(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def mode_code(mode: str) -> int:
    try:
        return _MODES[mode]
    except KeyError:
        raise ValueError(f"mode must be one of {sorted(_MODES)}, got {mode!r}") from None


class _Workspaces:
    """Zero-initialised scratch, one per (device, stream, host thread, kind), grown on demand.

    The kernels that need zeroed scratch (the surrogate's last-arriver ticket)
    leave it zeroed again, so a workspace is cleared only when it is created. Keyed by
    the host thread too: two threads enqueueing on one stream must not share scratch
    (their launches would interleave on it).
    """

    def __init__(self):
        self._ws: dict = {}
        self._pinned: dict = {}

    def get(self, device: torch.device, kind: str, nbytes: int, stream: int | None = None) -> torch.Tensor:
        key = (device.index, torch.cuda.current_stream(device).cuda_stream if stream is None else stream,
               threading.get_ident(), kind)
        t = self._ws.get(key)
        if t is None or t.numel() < nbytes:
            t = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=device)
            self._ws[key] = t
        return t

    def pinned(self, device: torch.device, stream: int) -> torch.Tensor:
        """16 page-locked int64 host words (the blocking evaluation's readback), same keying."""
        key = (device.index, stream, threading.get_ident())
        t = self._pinned.get(key)
        if t is None:
            t = self._pinned[key] = torch.zeros(16, dtype=torch.int64, pin_memory=True)
        return t


workspaces = _Workspaces()


def _label_code(y: torch.Tensor, name: str = "y") -> int:
    _require_gpu(y, name)
    try:
        return _LABEL_CODES[y.dtype]
    except KeyError:
        raise TypeError(f"{name} must be int8, int32 or int64, got {y.dtype}") from None


def _check_vec(h: torch.Tensor, y: torch.Tensor) -> int:
    _require(h, "h", torch.float32)
    if h.dim() != 1 or y.dim() != 1 or h.shape[0] != y.shape[0]:
        raise ValueError(f"h and y must be 1-D of equal length, got {tuple(h.shape)} and {tuple(y.shape)}")
    if y.stride(0) != 1:
        raise ValueError("y must be contiguous")
    if h.device != y.device:
        raise ValueError("h and y must be on the same device")
    if h.shape[0] == 0:
        raise ValueError("empty batch")
    return h.shape[0]


# ----------------------------------------------------------------- a1
def label_map_phat(labels: torch.Tensor, split_index: int, y_out: torch.Tensor, lcounts: torch.Tensor,
                   gcounts: torch.Tensor, p_hat: torch.Tensor) -> None:
    """main.py:303-310 in one launch: y_out = +/-1 (int8), lcounts += counts, p_hat (fp32)."""
    _require(labels, "labels", torch.int64)
    dev = labels.device
    _require(y_out, "y_out", torch.int8, dev)
    for t, n in ((lcounts, "lcounts"), (gcounts, "gcounts"), (p_hat, "p_hat")):
        _require(t, n, torch.float32, dev)
    if labels.dim() != 1 or not labels.is_contiguous() or y_out.shape != labels.shape or not y_out.is_contiguous():
        raise ValueError("labels and y_out must be contiguous 1-D tensors of equal length")
    if lcounts.numel() < 2 or gcounts.numel() < 2 or p_hat.numel() < 1 or labels.numel() == 0:
        raise ValueError("lcounts/gcounts need 2 elements, p_hat 1, labels >= 1")
    check(_lib.load().dauc_label_map_phat(_ptr(labels), labels.numel(), int(split_index), _ptr(y_out),
                                          _ptr(lcounts), _ptr(gcounts), _ptr(p_hat), _stream(dev)),
          "dauc_label_map_phat")


# ----------------------------------------------------------------- a2/a3
def surrogate_fwdbwd(h: torch.Tensor, y: torch.Tensor, abalpha: torch.Tensor, p_hat: torch.Tensor, *,
                     dh: torch.Tensor | None = None, out64: torch.Tensor | None = None,
                     grad3: torch.Tensor | None = None, loss: torch.Tensor | None = None,
                     variant: int = 0) -> None:
    """Fused loss + gradients of main.py:313-317 (one pass over h and y).

    ``variant`` != 0 runs a measured alternative from the tuning build (include/dauc_tuning.h:
    1 persistent kernel, 2 two-launch form, 3 stream alone, 20 the one-launch kernel at any unit-stride
    B, 22 its stream with the row stores and no reduce, 23 variant 20 with one row never published:
    the timeout path, for tests). ``surrogate_status`` reports a timed-out reduction."""
    B = _check_vec(h, y)
    dev = h.device
    yc = _label_code(y)
    _require(abalpha, "abalpha", torch.float32, dev)
    _require(p_hat, "p_hat", torch.float32, dev)
    if abalpha.numel() < 3 or not abalpha.is_contiguous() or p_hat.numel() < 1:
        raise ValueError("abalpha needs 3 contiguous fp32 values, p_hat 1")
    dh_stride = 1
    if dh is not None:
        _require(dh, "dh", torch.float32, dev)
        if dh.dim() != 1 or dh.shape[0] != B:
            raise ValueError("dh must be 1-D of length B")
        dh_stride = dh.stride(0)
    if out64 is not None:
        _require(out64, "out64", torch.float64, dev)
        if out64.numel() < 6 or not out64.is_contiguous():
            raise ValueError("out64 needs 6 contiguous fp64 slots")
    if grad3 is not None:
        _require(grad3, "grad3", torch.float32, dev)
        if grad3.numel() < 3 or not grad3.is_contiguous():
            raise ValueError("grad3 needs 3 contiguous fp32 slots")
    if loss is not None:
        _require(loss, "loss", torch.float32, dev)
    # variants run in the tuning build, whose workspace also holds the stamp region
    L = _lib.load() if variant == 0 else _lib.tuning()
    nbytes = L.dauc_surrogate_workspace_size(B)
    ws = workspaces.get(dev, "surrogate" if variant == 0 else "surrogate_tuning", nbytes)
    if variant == 0:
        rc = L.dauc_surrogate_fwdbwd(_ptr(h), h.stride(0), _ptr(y), yc, B, _ptr(abalpha), _ptr(p_hat),
                                     _ptr(dh), dh_stride, _ptr(out64), _ptr(grad3), _ptr(loss), _ptr(ws),
                                     ws.numel(), _stream(dev))
    else:
        rc = L.dauc_surrogate_fwdbwd_variant(_ptr(h), h.stride(0), _ptr(y), yc, B, _ptr(abalpha), _ptr(p_hat),
                                             _ptr(dh), dh_stride, _ptr(out64), _ptr(grad3), _ptr(loss), _ptr(ws),
                                             ws.numel(), int(variant), _stream(dev))
    check(rc, "dauc_surrogate_fwdbwd")


SURROGATE_TIMEOUT = 1  # dauc_surrogate_status bit 0


def surrogate_status(device, *, clear: bool = True, variant: int = 0, raise_on_error: bool = False) -> int:
    """The sticky status word of this stream's loss workspace (dauc_surrogate_status: a BLOCKING
    read). 0 = every loss call since the last clear completed its reduction; bit 0 = a reducer of
    the one-launch loss (B >= 2^22) timed out and that call returned NaN -- a failed reduction, not
    a diverged loss. ``raise_on_error`` raises DaucError instead of returning a nonzero word."""
    dev = torch.device(device)
    L = _lib.load() if variant == 0 else _lib.tuning()
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream, threading.get_ident(),
           "surrogate" if variant == 0 else "surrogate_tuning")
    ws = workspaces._ws.get(key)
    if ws is None:
        return 0  # no loss call on this stream yet
    out = ctypes.c_uint(0)
    check(L.dauc_surrogate_status(_ptr(ws), ws.numel(), ctypes.byref(out), int(bool(clear)), _stream(dev)),
          "dauc_surrogate_status")
    if raise_on_error and out.value:
        raise _lib.DaucError(f"dauc_surrogate_fwdbwd: a reducer of the one-launch loss timed out (status "
                             f"{out.value:#x}); the affected call's loss and gradients are NaN")
    return out.value


def class_sums(h: torch.Tensor, y: torch.Tensor, sums4: torch.Tensor, accumulate: bool = True) -> None:
    """main.py:185-188: sums4 (+)= {sum h[y=-1], #neg, sum h[y=1], #pos} (fp64)."""
    B = _check_vec(h, y)
    dev = h.device
    yc = _label_code(y)
    _require(sums4, "sums4", torch.float64, dev)
    if sums4.numel() < 4 or not sums4.is_contiguous():
        raise ValueError("sums4 needs 4 contiguous fp64 slots")
    L = _lib.load()
    ws = workspaces.get(dev, "surrogate", L.dauc_surrogate_workspace_size(B))
    check(L.dauc_class_sums(_ptr(h), h.stride(0), _ptr(y), yc, B, _ptr(sums4), int(bool(accumulate)),
                            _ptr(ws), ws.numel(), _stream(dev)), "dauc_class_sums")


_Z_CODES = {torch.float32: _lib.DTYPE_F32, torch.bfloat16: _lib.DTYPE_BF16}


def _check_logits(z: torch.Tensor, y: torch.Tensor) -> tuple[int, int]:
    _require_gpu(z, "z")
    if z.dtype not in _Z_CODES:
        raise TypeError(f"logits must be fp32 or bf16, got {z.dtype}")
    if z.dim() != 2 or z.shape[1] != 2 or z.stride(1) != 1:
        raise ValueError(f"logits must be [B, 2] with unit column stride, got {tuple(z.shape)} {z.stride()}")
    if y.dim() != 1 or y.shape[0] != z.shape[0] or y.stride(0) != 1 or y.device != z.device:
        raise ValueError("labels must be contiguous [B] on the logits' device")
    if z.shape[0] == 0:
        raise ValueError("empty batch")
    return z.shape[0], _Z_CODES[z.dtype]


def surrogate_logits_fwdbwd(z: torch.Tensor, y: torch.Tensor, abalpha: torch.Tensor, p_hat: torch.Tensor, *,
                            dz: torch.Tensor | None = None, h_out: torch.Tensor | None = None,
                            out64: torch.Tensor | None = None, grad3: torch.Tensor | None = None,
                            loss: torch.Tensor | None = None) -> None:
    """loss and dF/dz straight from the [B,2] logits (softmax column fused)."""
    B, zc = _check_logits(z, y)
    dev = z.device
    yc = _label_code(y)
    _require(abalpha, "abalpha", torch.float32, dev)
    _require(p_hat, "p_hat", torch.float32, dev)
    if abalpha.numel() < 3 or not abalpha.is_contiguous():
        raise ValueError("abalpha needs 3 contiguous fp32 values")
    lddz = 2
    if dz is not None:
        _require(dz, "dz", z.dtype, dev)
        if dz.shape != z.shape or dz.stride(1) != 1:
            raise ValueError("dz must match the logits' shape with unit column stride")
        lddz = dz.stride(0)
    if h_out is not None:
        _require(h_out, "h_out", torch.float32, dev)
        if h_out.numel() < B or not h_out.is_contiguous():
            raise ValueError("h_out needs B contiguous fp32 slots")
    for t, n, dt, k in ((out64, "out64", torch.float64, 6), (grad3, "grad3", torch.float32, 3)):
        if t is not None:
            _require(t, n, dt, dev)
            if t.numel() < k or not t.is_contiguous():
                raise ValueError(f"{n} needs {k} contiguous slots")
    if loss is not None:
        _require(loss, "loss", torch.float32, dev)
    L = _lib.load()
    ws = workspaces.get(dev, "surrogate", L.dauc_surrogate_workspace_size(B))
    check(L.dauc_surrogate_logits_fwdbwd(_ptr(z), zc, z.stride(0), _ptr(y), yc, B, _ptr(abalpha), _ptr(p_hat),
                                         _ptr(dz), lddz, _ptr(h_out), _ptr(out64), _ptr(grad3), _ptr(loss),
                                         _ptr(ws), ws.numel(), _stream(dev)), "dauc_surrogate_logits_fwdbwd")


def class_sums_logits(z: torch.Tensor, y: torch.Tensor, sums4: torch.Tensor, accumulate: bool = True,
                      h_out: torch.Tensor | None = None) -> None:
    """class_sums with h = softmax(z)[:, 1] computed in the kernel."""
    B, zc = _check_logits(z, y)
    dev = z.device
    yc = _label_code(y)
    _require(sums4, "sums4", torch.float64, dev)
    if h_out is not None:
        _require(h_out, "h_out", torch.float32, dev)
    L = _lib.load()
    ws = workspaces.get(dev, "surrogate", L.dauc_surrogate_workspace_size(B))
    check(L.dauc_class_sums_logits(_ptr(z), zc, z.stride(0), _ptr(y), yc, B, _ptr(h_out), _ptr(sums4),
                                   int(bool(accumulate)), _ptr(ws), ws.numel(), _stream(dev)),
          "dauc_class_sums_logits")


def alpha_from_sums(sums4: torch.Tensor, alpha: torch.Tensor) -> None:
    """main.py:197 on the device: alpha = h_neg/N_neg - h_pos/N_pos."""
    _require(sums4, "sums4", torch.float64)
    _require(alpha, "alpha", torch.float32, sums4.device)
    check(_lib.load().dauc_alpha_from_sums(_ptr(sums4), _ptr(alpha), _stream(sums4.device)),
          "dauc_alpha_from_sums")


# ----------------------------------------------------------------- a4/a5
def pd_update(w: torch.Tensor, w0: torch.Tensor, w_avg: torch.Tensor | None, segs, nseg: int, *,
              scalars: torch.Tensor | None = None, grad3: torch.Tensor | None = None,
              anchor3: torch.Tensor | None = None, lr: float, gamma: float, mode: str = "reference") -> None:
    """dppd_sg over the flat buffer + running average, one launch (segs: GradSeg ctypes array).

    The caller guarantees every segment lies inside w / w0 / w_avg (FlatState builds
    the table from the parameters' own offsets).
    """
    _require(w, "w", torch.float32)
    dev = w.device
    _require(w0, "w0", torch.float32, dev)
    if w_avg is not None:
        _require(w_avg, "w_avg", torch.float32, dev)
    if scalars is not None:
        for t, n in ((scalars, "scalars"), (grad3, "grad3"), (anchor3, "anchor3")):
            _require(t, n, torch.float32, dev)
    check(_lib.load().dauc_pd_update(_ptr(w), _ptr(w0), _ptr(w_avg), segs, int(nseg), _ptr(scalars),
                                     _ptr(grad3), _ptr(anchor3), float(lr), float(1 / gamma),
                                     mode_code(mode), _stream(dev)),
          "dauc_pd_update")


def pd_update_dense(w: torch.Tensor, g: torch.Tensor, w0: torch.Tensor, w_avg: torch.Tensor | None, *,
                    lr: float, gamma: float, variant: int = 0) -> None:
    """main.py:61 (+333-334) over one dense buffer of n parameters."""
    _require(w, "w", torch.float32)
    dev = w.device
    n = w.numel()
    for t, name in ((g, "g"), (w0, "w0")) + (((w_avg, "w_avg"),) if w_avg is not None else ()):
        _require(t, name, torch.float32, dev)
        if t.numel() != n or not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous with {n} elements")
    if not w.is_contiguous():
        raise ValueError("w must be contiguous")
    if variant == 0:
        rc = _lib.load().dauc_pd_update_dense(_ptr(w), _ptr(g), _ptr(w0), _ptr(w_avg), n, float(lr),
                                              float(1 / gamma), _stream(dev))
    else:  # a measured alternative geometry (tuning build)
        rc = _lib.tuning().dauc_pd_update_dense_variant(_ptr(w), _ptr(g), _ptr(w0), _ptr(w_avg), n, float(lr),
                                                        float(1 / gamma), int(variant), _stream(dev))
    check(rc, "dauc_pd_update_dense")


# ----------------------------------------------------------------- a6
def coda_finalize(flat: torch.Tensor, n_avg: int, world: int, lcounts: torch.Tensor,
                  gcounts: torch.Tensor) -> None:
    """Divide the all-reduced flat[:n_avg] by world and fold the class counts."""
    _require(flat, "flat", torch.float32)
    dev = flat.device
    _require(lcounts, "lcounts", torch.float32, dev)
    _require(gcounts, "gcounts", torch.float32, dev)
    if not flat.is_contiguous() or n_avg > flat.numel() or n_avg < 0:
        raise ValueError("flat must be contiguous and hold n_avg elements")
    check(_lib.load().dauc_coda_finalize(_ptr(flat), int(n_avg), int(world), _ptr(lcounts), _ptr(gcounts),
                                         _stream(dev)), "dauc_coda_finalize")


def scale_div(x: torch.Tensor, divisor: float) -> None:
    """x /= divisor (fp32 IEEE division), main.py:338-339."""
    _require(x, "x", torch.float32)
    if not x.is_contiguous():
        raise ValueError("x must be contiguous")
    check(_lib.load().dauc_scale_div(_ptr(x), x.numel(), float(divisor), _stream(x.device)), "dauc_scale_div")


# ----------------------------------------------------------------- a8
def split_scores(scores: torch.Tensor, labels: torch.Tensor, negatives: bool = True):
    """Stable split into (pos, neg) score buffers plus device stats {P, N, non-finite, other}.

    Returns (pos_buf, neg_buf, stats): pos_buf/neg_buf have capacity n; the valid
    prefixes are stats[0] and stats[1] long. negatives=False writes only the
    positives (neg_buf is None).
    """
    _require(scores, "scores", torch.float32)
    dev = scores.device
    lc = _label_code(labels, "labels")
    if scores.dim() != 1 or labels.dim() != 1 or scores.shape != labels.shape:
        raise ValueError("scores and labels must be 1-D of equal length")
    if not scores.is_contiguous() or not labels.is_contiguous():
        raise ValueError("scores and labels must be contiguous")
    n = scores.numel()
    if n == 0:
        raise ValueError("empty score vector")
    pos = torch.empty(n, dtype=torch.float32, device=dev)
    neg = torch.empty(n, dtype=torch.float32, device=dev) if negatives else None
    stats = torch.empty(4, dtype=torch.int64, device=dev)
    L = _lib.load()
    ws = workspaces.get(dev, "split", L.dauc_split_workspace_size(n))
    check(L.dauc_split_scores(_ptr(scores), _ptr(labels), lc, n, _ptr(pos), _ptr(neg) if negatives else None,
                              _ptr(stats), _ptr(ws), ws.numel(), _stream(dev)), "dauc_split_scores")
    return pos, neg, stats


def _eval_args(scores: torch.Tensor, labels: torch.Tensor):
    _require(scores, "scores", torch.float32)
    dev = scores.device
    lc = _label_code(labels, "labels")
    if scores.dim() != 1 or labels.dim() != 1 or scores.shape != labels.shape:
        raise ValueError("scores and labels must be 1-D of equal length")
    if not scores.is_contiguous() or not labels.is_contiguous():
        raise ValueError("scores and labels must be contiguous")
    n = scores.numel()
    if n == 0:
        raise ValueError("empty score vector")
    L = _lib.load()
    # keyed by library too: the tuning build's evaluation workspace also holds its range-slot path
    nbytes = _eval_ws_bytes.get((id(L), n))
    if nbytes is None:
        nbytes = _eval_ws_bytes[(id(L), n)] = L.dauc_auc_eval_workspace_size(n)
    st = torch.cuda.current_stream(dev).cuda_stream
    return L, dev, lc, n, st, workspaces.get(dev, "auc_eval", nbytes, st)


def auc_eval_counts(scores: torch.Tensor, labels: torch.Tensor) -> tuple:
    """The single-GPU sort-method evaluation in one blocking ABI call (dauc_auc_eval_counts):
    (W, T, P, N, #non-finite scores, #labels not in {-1, 1}) as Python ints."""
    L, dev, lc, n, st, ws = _eval_args(scores, labels)
    pin = workspaces.pinned(dev, st)
    out = (ctypes.c_int64 * 6)()
    check(L.dauc_auc_eval_counts(scores.data_ptr(), labels.data_ptr(), lc, n, ctypes.addressof(out), pin.data_ptr(),
                                 ws.data_ptr(), ws.numel(), st), "dauc_auc_eval_counts")
    return tuple(out)


def auc_eval_enqueue(scores: torch.Tensor, labels: torch.Tensor, part: int, parts: int,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """Part `part` of `parts` of the evaluation, enqueued with no host synchronisation
    (dauc_auc_eval_enqueue). Returns the device int64 [8] record: W_part, T_part, #non-finite
    queried scores (sum these over the parts), P, 0, #non-finite positives, #labels not in
    {-1, 1}, verdict (1 counted, 0 empty part, 2 run the blocking sorted path)."""
    L, dev, lc, n, st, ws = _eval_args(scores, labels)
    if out is None:
        out = torch.empty(8, dtype=torch.int64, device=dev)
    elif out.dtype != torch.int64 or out.numel() < 8 or not out.is_contiguous() or out.device != dev:
        raise ValueError("out must be a contiguous int64 tensor of >= 8 elements on the scores' device")
    check(L.dauc_auc_eval_enqueue(scores.data_ptr(), labels.data_ptr(), lc, n, int(part), int(parts), out.data_ptr(),
                                  ws.data_ptr(), ws.numel(), st), "dauc_auc_eval_enqueue")
    return out


def auc_slot_bytes(n: int, parts: int) -> int:
    """Bytes of one rank's slot of the two-step sharded evaluation (dauc_auc_slot_bytes)."""
    return int(_lib.load().dauc_auc_slot_bytes(int(n), int(parts)))


def auc_eval_compact_part(scores: torch.Tensor, labels: torch.Tensor, part: int, parts: int,
                          slot: torch.Tensor) -> torch.Tensor:
    """Step 1 of the two-step sharded evaluation (dauc_auc_eval_compact_part): this rank's slice
    of the labels compacted into `slot` (a contiguous uint8 tensor of auc_slot_bytes(n, parts)
    bytes, 256-byte aligned, on the scores' device), enqueued with no host synchronisation."""
    L, dev, lc, n, st, ws = _eval_args(scores, labels)
    nb = auc_slot_bytes(n, parts)
    if (slot.dtype != torch.uint8 or slot.numel() < nb or not slot.is_contiguous() or slot.device != dev
            or slot.data_ptr() % 256):
        raise ValueError(f"slot must be a contiguous, 256-byte aligned uint8 tensor of >= {nb} bytes on the scores' device")
    check(L.dauc_auc_eval_compact_part(scores.data_ptr(), labels.data_ptr(), lc, n, int(part), int(parts),
                                       slot.data_ptr(), ws.data_ptr(), ws.numel(), st), "dauc_auc_eval_compact_part")
    return slot


def auc_eval_query_part(scores: torch.Tensor, labels: torch.Tensor, part: int, parts: int, slots: torch.Tensor,
                        out: torch.Tensor | None = None) -> torch.Tensor:
    """Step 2 (dauc_auc_eval_query_part): the `parts` gathered slots (contiguous, rank order) become
    the positive table; this rank's query range is counted. Returns the device int64 [8] record of
    auc_eval_enqueue (verdict 2: every rank runs the blocking sorted path)."""
    L, dev, lc, n, st, ws = _eval_args(scores, labels)
    nb = auc_slot_bytes(n, parts)
    if (slots.dtype != torch.uint8 or slots.numel() < nb * int(parts) or not slots.is_contiguous()
            or slots.device != dev or slots.data_ptr() % 256):
        raise ValueError("slots must be the contiguous, 256-byte aligned uint8 gather of every rank's slot")
    if out is None:
        out = torch.empty(8, dtype=torch.int64, device=dev)
    elif out.dtype != torch.int64 or out.numel() < 8 or not out.is_contiguous() or out.device != dev:
        raise ValueError("out must be a contiguous int64 tensor of >= 8 elements on the scores' device")
    check(L.dauc_auc_eval_query_part(scores.data_ptr(), labels.data_ptr(), lc, n, int(part), int(parts),
                                     slots.data_ptr(), out.data_ptr(), ws.data_ptr(), ws.numel(), st),
          "dauc_auc_eval_query_part")
    return out


def auc_eval_query_part_sorted(scores: torch.Tensor, labels: torch.Tensor, part: int, parts: int,
                               slots: torch.Tensor, P: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """The two-step evaluation's verdict-2 path (dauc_auc_eval_query_part_sorted): the gathered
    slots' P positives sorted into one table (the distinct-key index for tie-heavy tables, else the
    LDS tree), this rank's own slice counted. Returns the device int64 [8] record {W, T, #non-finite
    queried, P, 0, 0, 0, verdict}; verdict 2: a slot overflowed (or P > n - P) -- run
    auc_eval_counts_part instead."""
    L, dev, lc, n, st, ws = _eval_args(scores, labels)
    nb = auc_slot_bytes(n, parts)
    if (slots.dtype != torch.uint8 or slots.numel() < nb * int(parts) or not slots.is_contiguous()
            or slots.device != dev or slots.data_ptr() % 256):
        raise ValueError("slots must be the contiguous, 256-byte aligned uint8 gather of every rank's slot")
    if out is None:
        out = torch.empty(8, dtype=torch.int64, device=dev)
    elif out.dtype != torch.int64 or out.numel() < 8 or not out.is_contiguous() or out.device != dev:
        raise ValueError("out must be a contiguous int64 tensor of >= 8 elements on the scores' device")
    check(L.dauc_auc_eval_query_part_sorted(scores.data_ptr(), labels.data_ptr(), lc, n, int(part), int(parts),
                                            slots.data_ptr(), int(P), out.data_ptr(), ws.data_ptr(), ws.numel(), st),
          "dauc_auc_eval_query_part_sorted")
    return out


def auc_eval_counts_part(scores: torch.Tensor, labels: torch.Tensor, part: int, parts: int,
                         part_counts: torch.Tensor) -> tuple:
    """Part `part` of `parts` of the blocking evaluation (dauc_auc_eval_counts_part): every part
    builds the table from all the positives, only the queries are split. Returns (W_part, T_part,
    P, N, #non-finite positives, #labels not in {-1, 1}, #non-finite queried scores of this part);
    `part_counts` (int64 [3] on the device) receives (W_part, T_part, that last count) on the
    current stream for an all-reduce."""
    _require(part_counts, "part_counts", torch.int64)
    L, dev, lc, n, st, ws = _eval_args(scores, labels)
    if part_counts.numel() < 3 or not part_counts.is_contiguous() or part_counts.device != dev:
        raise ValueError("part_counts must be a contiguous int64 tensor of >= 3 elements on the scores' device")
    pin = workspaces.pinned(dev, st)
    out = (ctypes.c_int64 * 7)()
    check(L.dauc_auc_eval_counts_part(scores.data_ptr(), labels.data_ptr(), lc, n, int(part), int(parts),
                                      ctypes.addressof(out), part_counts.data_ptr(), pin.data_ptr(), ws.data_ptr(),
                                      ws.numel(), st), "dauc_auc_eval_counts_part")
    return tuple(out)


_eval_ws_bytes: dict = {}  # dauc_auc_eval_workspace_size per (library, length) (a pure function of n)


def compact_positives(scores: torch.Tensor, labels: torch.Tensor):
    """Positive scores (label == 1) in original order, reading only the labels and the positives' scores.

    Returns (pos_buf, stats): pos_buf has capacity n, its valid prefix is stats[0] long;
    stats (device int64 [4]) = {P, n - P, #non-finite positive scores, #labels not in {-1, 1}}.
    """
    _require(scores, "scores", torch.float32)
    dev = scores.device
    lc = _label_code(labels, "labels")
    if scores.dim() != 1 or labels.dim() != 1 or scores.shape != labels.shape:
        raise ValueError("scores and labels must be 1-D of equal length")
    if not scores.is_contiguous() or not labels.is_contiguous():
        raise ValueError("scores and labels must be contiguous")
    n = scores.numel()
    if n == 0:
        raise ValueError("empty score vector")
    pos = torch.empty(n, dtype=torch.float32, device=dev)
    stats = torch.empty(4, dtype=torch.int64, device=dev)
    L = _lib.load()
    ws = workspaces.get(dev, "compact", L.dauc_compact_workspace_size(n))
    check(L.dauc_compact_positives(_ptr(scores), _ptr(labels), lc, n, _ptr(pos), _ptr(stats), _ptr(ws),
                                   ws.numel(), _stream(dev)), "dauc_compact_positives")
    return pos, stats


def pair_count(pos: torch.Tensor, neg: torch.Tensor, wins_ties: torch.Tensor, variant: int = 0) -> None:
    """wins_ties[0] += #{pos > neg}, wins_ties[1] += #{pos == neg} (int64 view of uint64 counters)."""
    _require(pos, "pos", torch.float32)
    dev = pos.device
    _require(neg, "neg", torch.float32, dev)
    _require(wins_ties, "wins_ties", torch.int64, dev)
    if pos.dim() != 1 or neg.dim() != 1 or not pos.is_contiguous() or not neg.is_contiguous():
        raise ValueError("pos and neg must be contiguous 1-D tensors")
    if wins_ties.numel() < 2 or not wins_ties.is_contiguous():
        raise ValueError("wins_ties needs 2 contiguous int64 slots")
    if variant == 0:
        rc = _lib.load().dauc_pair_count(_ptr(pos), pos.numel(), _ptr(neg), neg.numel(), _ptr(wins_ties),
                                         _stream(dev))
    else:  # a measured alternative counting scheme (tuning build)
        rc = _lib.tuning().dauc_pair_count_variant(_ptr(pos), pos.numel(), _ptr(neg), neg.numel(), _ptr(wins_ties),
                                                   int(variant), _stream(dev))
    check(rc, "dauc_pair_count")


def auc_counts_sorted(pos: torch.Tensor, neg: torch.Tensor, wins_ties: torch.Tensor) -> None:
    """Same (wins, ties) accumulation as pair_count, by radix-sorting the smaller class and
    locating every score of the larger one in it (LDS search tree + one bucket load)."""
    _require(pos, "pos", torch.float32)
    dev = pos.device
    _require(neg, "neg", torch.float32, dev)
    _require(wins_ties, "wins_ties", torch.int64, dev)
    if pos.dim() != 1 or neg.dim() != 1 or not pos.is_contiguous() or not neg.is_contiguous():
        raise ValueError("pos and neg must be contiguous 1-D tensors")
    if wins_ties.numel() < 2 or not wins_ties.is_contiguous():
        raise ValueError("wins_ties needs 2 contiguous int64 slots")
    L = _lib.load()
    ws = workspaces.get(dev, "sort", L.dauc_sort_workspace_size(max(min(pos.numel(), neg.numel()), 1)))
    check(L.dauc_auc_counts_sorted(_ptr(pos), pos.numel(), _ptr(neg), neg.numel(), _ptr(wins_ties), _ptr(ws),
                                   ws.numel(), _stream(dev)), "dauc_auc_counts_sorted")


def auc_counts_sorted_labeled(pos: torch.Tensor, scores: torch.Tensor, labels: torch.Tensor, begin: int, end: int,
                              wins_ties: torch.Tensor, nonfinite: torch.Tensor | None = None) -> None:
    """auc_counts_sorted with the negatives read in place: every element of scores[begin:end]
    whose label is not 1 is counted against the sorted positives; nonfinite (int64 [1],
    optional) += the number of those scores that are NaN or infinite."""
    _require(pos, "pos", torch.float32)
    dev = pos.device
    _require(scores, "scores", torch.float32, dev)
    _require(wins_ties, "wins_ties", torch.int64, dev)
    lc = _label_code(labels, "labels")
    if pos.dim() != 1 or not pos.is_contiguous() or scores.dim() != 1 or not scores.is_contiguous():
        raise ValueError("pos and scores must be contiguous 1-D tensors")
    if labels.shape != scores.shape or not labels.is_contiguous() or labels.device != dev:
        raise ValueError("labels must be a contiguous tensor shaped like scores, on the same device")
    if not 0 <= begin <= end <= scores.numel():
        raise ValueError("need 0 <= begin <= end <= scores.numel()")
    if wins_ties.numel() < 2 or not wins_ties.is_contiguous():
        raise ValueError("wins_ties needs 2 contiguous int64 slots")
    if nonfinite is not None:
        _require(nonfinite, "nonfinite", torch.int64, dev)
        if nonfinite.numel() < 1:
            raise ValueError("nonfinite needs 1 int64 slot")
    L = _lib.load()
    ws = workspaces.get(dev, "sort", L.dauc_sort_workspace_size(max(pos.numel(), 1)))
    check(L.dauc_auc_counts_sorted_labeled(_ptr(pos), pos.numel(), _ptr(scores), _ptr(labels), lc, int(begin),
                                           int(end), _ptr(wins_ties), _ptr(nonfinite), _ptr(ws), ws.numel(),
                                           _stream(dev)),
          "dauc_auc_counts_sorted_labeled")


def sort_keys(scores: torch.Tensor) -> torch.Tensor:
    """Ascending order-preserving uint32 keys of fp32 scores, returned as int32 bit patterns."""
    _require(scores, "scores", torch.float32)
    if scores.dim() != 1 or not scores.is_contiguous() or scores.numel() == 0:
        raise ValueError("scores must be a non-empty contiguous 1-D tensor")
    dev = scores.device
    out = torch.empty(scores.numel(), dtype=torch.int32, device=dev)
    L = _lib.load()
    ws = workspaces.get(dev, "sort", L.dauc_sort_workspace_size(scores.numel()))
    check(L.dauc_sort_keys(_ptr(scores), scores.numel(), _ptr(out), _ptr(ws), ws.numel(), _stream(dev)),
          "dauc_sort_keys")
    return out


def conv3x3_wgrad(x: torch.Tensor, dy: torch.Tensor, stride: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """The fp32 weight gradient of a 3x3 / pad 1 / stride 1|2 convolution from its channels-last
    bf16 input x [N, Ci, H, W] and output gradient dy [N, Co, Ho, Wo] (dauc_conv3x3_wgrad):
    a [Co, Ci, 3, 3] fp32 tensor in channels-last memory order (the backbone's parameter layout)."""
    _require(x, "x", torch.bfloat16)
    _require(dy, "dy", torch.bfloat16, x.device)
    if x.dim() != 4 or dy.dim() != 4 or x.shape[0] != dy.shape[0]:
        raise ValueError(f"x and dy must be [N, C, H, W] of one batch, got {tuple(x.shape)} and {tuple(dy.shape)}")
    for t, name in ((x, "x"), (dy, "dy")):
        if not t.is_contiguous(memory_format=torch.channels_last):
            raise ValueError(f"{name} must be channels-last contiguous")
    N, Ci, H, W = x.shape
    Co, Ho, Wo = dy.shape[1], dy.shape[2], dy.shape[3]
    dev = x.device
    if out is None:
        out = torch.empty((Co, Ci, 3, 3), dtype=torch.float32, device=dev, memory_format=torch.channels_last)
    elif (out.dtype != torch.float32 or tuple(out.shape) != (Co, Ci, 3, 3)
          or not out.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("out must be a channels-last fp32 [Co, Ci, 3, 3] tensor")
    L = _lib.load()
    nbytes = L.dauc_conv3x3_wgrad_workspace_size(N, Ho, Wo, Ci, Co)
    ws = workspaces.get(dev, "wgrad3x3", nbytes) if nbytes else None
    check(L.dauc_conv3x3_wgrad(_ptr(x), _ptr(dy), _lib.DTYPE_BF16, N, H, W, Ci, Ho, Wo, Co, int(stride), _ptr(out),
                               _ptr(ws), 0 if ws is None else ws.numel(), _stream(dev)), "dauc_conv3x3_wgrad")
    return out


def conv3x3_wgrad_supported(x: torch.Tensor, dy: torch.Tensor, stride, padding, dilation, groups) -> bool:
    """The shapes dauc_conv3x3_wgrad takes (the ResNet bottlenecks' and basic blocks' 3x3 convolutions)."""
    s = tuple(stride) if isinstance(stride, (tuple, list)) else (stride, stride)
    p = tuple(padding) if isinstance(padding, (tuple, list)) else (padding, padding)
    d = tuple(dilation) if isinstance(dilation, (tuple, list)) else (dilation, dilation)
    return (x.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16 and x.is_cuda and groups == 1
            and s[0] == s[1] and s[0] in (1, 2) and p == (1, 1) and d == (1, 1)
            and x.shape[1] % 64 == 0 and dy.shape[1] % 64 == 0
            and x.is_contiguous(memory_format=torch.channels_last)
            and dy.is_contiguous(memory_format=torch.channels_last)
            and x.shape[0] * x.shape[2] * x.shape[3] < 2 ** 31)


def _stem_shapes(x: torch.Tensor):
    _require(x, "x", torch.bfloat16)
    if x.dim() != 4 or x.shape[1] != 3 or not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError(f"x must be a channels-last [N, 3, H, W] bf16 tensor, got {tuple(x.shape)}")
    if x.data_ptr() % 16:
        raise ValueError("x must be 16-byte aligned")
    N, _, H, W = x.shape
    return N, H, W, (H - 1) // 2 + 1, (W - 1) // 2 + 1


def stem_conv_forward(x: torch.Tensor, weight: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """conv2d(x, weight, stride=2, padding=3) for the 7x7 stem (resnet.py:145) on channels-last bf16
    (dauc_conv7x7s2_stem_forward): x [N, 3, H, W], weight [64, 3, 7, 7] bf16 in channels-last
    memory order; returns a channels-last bf16 [N, 64, Ho, Wo]."""
    N, H, W, Ho, Wo = _stem_shapes(x)
    _require(weight, "weight", torch.bfloat16, x.device)
    if tuple(weight.shape) != (64, 3, 7, 7) or not weight.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("weight must be a channels-last bf16 [64, 3, 7, 7] tensor")
    if out is None:
        out = torch.empty((N, 64, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    elif (out.dtype != torch.bfloat16 or tuple(out.shape) != (N, 64, Ho, Wo)
          or not out.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("out must be a channels-last bf16 [N, 64, Ho, Wo] tensor")
    check(_lib.load().dauc_conv7x7s2_stem_forward(_ptr(x), _ptr(weight), _lib.DTYPE_BF16, N, H, W, Ho, Wo, _ptr(out),
                                                  _stream(x.device)), "dauc_conv7x7s2_stem_forward")
    return out


def stem_conv_wgrad(x: torch.Tensor, dy: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """The fp32 weight gradient of the 7x7 / stride-2 / pad-3 stem from its channels-last bf16 input
    x [N, 3, H, W] and output gradient dy [N, 64, Ho, Wo] (dauc_conv7x7s2_stem_wgrad): a [64, 3, 7, 7]
    fp32 tensor in channels-last memory order (the backbone's parameter layout)."""
    N, H, W, Ho, Wo = _stem_shapes(x)
    _require(dy, "dy", torch.bfloat16, x.device)
    if tuple(dy.shape) != (N, 64, Ho, Wo) or not dy.is_contiguous(memory_format=torch.channels_last):
        raise ValueError(f"dy must be a channels-last bf16 [{N}, 64, {Ho}, {Wo}] tensor, got {tuple(dy.shape)}")
    dev = x.device
    if out is None:
        out = torch.empty((64, 3, 7, 7), dtype=torch.float32, device=dev, memory_format=torch.channels_last)
    elif (out.dtype != torch.float32 or tuple(out.shape) != (64, 3, 7, 7)
          or not out.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("out must be a channels-last fp32 [64, 3, 7, 7] tensor")
    L = _lib.load()
    nbytes = L.dauc_conv7x7s2_stem_wgrad_workspace_size(N, Ho, Wo)
    ws = workspaces.get(dev, "wgrad_stem", nbytes) if nbytes else None
    check(L.dauc_conv7x7s2_stem_wgrad(_ptr(x), _ptr(dy), _lib.DTYPE_BF16, N, H, W, Ho, Wo, _ptr(out), _ptr(ws),
                                      0 if ws is None else ws.numel(), _stream(dev)), "dauc_conv7x7s2_stem_wgrad")
    return out


def stem_conv_supported(x: torch.Tensor, weight: torch.Tensor, stride, padding, dilation, groups) -> bool:
    """The convolutions dauc_conv7x7s2_stem_* take: the ResNet stem on a channels-last bf16 image."""
    s = tuple(stride) if isinstance(stride, (tuple, list)) else (stride, stride)
    p = tuple(padding) if isinstance(padding, (tuple, list)) else (padding, padding)
    d = tuple(dilation) if isinstance(dilation, (tuple, list)) else (dilation, dilation)
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] == 3 and groups == 1
            and tuple(weight.shape) == (64, 3, 7, 7) and s == (2, 2) and p == (3, 3) and d == (1, 1)
            and x.is_contiguous(memory_format=torch.channels_last)
            # the kernels read a channels-last bf16 weight; an NCHW model (build_backbone's default)
            # fed channels-last images takes F.conv2d instead
            and weight.dtype == torch.bfloat16 and weight.is_contiguous(memory_format=torch.channels_last)):
        return False
    N, _, H, W = x.shape
    return (x.data_ptr() % 16 == 0 and N * H * W * 3 < 2 ** 31
            and (N * ((H - 1) // 2 + 1) * ((W - 1) // 2 + 1) + 128) * 64 < 2 ** 31)


def _cl_bf16(t: torch.Tensor, name: str) -> None:
    _require(t, name, torch.bfloat16)
    if t.dim() != 4 or not t.is_contiguous(memory_format=torch.channels_last) or t.shape[1] % 8 or t.data_ptr() % 16:
        raise ValueError(f"{name} must be a 16-byte aligned channels-last bf16 [N, C, H, W] tensor with C % 8 == 0")


def strided_pick(x: torch.Tensor, stride: int) -> torch.Tensor:
    """x[:, :, ::stride, ::stride] as a new channels-last tensor (dauc_strided_pick)."""
    _cl_bf16(x, "x")
    N, C, H, W = x.shape
    out = torch.empty((N, C, (H - 1) // stride + 1, (W - 1) // stride + 1), dtype=x.dtype, device=x.device,
                      memory_format=torch.channels_last)
    check(_lib.load().dauc_strided_pick(_ptr(x), _lib.DTYPE_BF16, N, H, W, C, int(stride), _ptr(out),
                                        _stream(x.device)), "dauc_strided_pick")
    return out


def strided_add_(dx: torch.Tensor, src: torch.Tensor, stride: int) -> torch.Tensor:
    """dx[:, :, ::stride, ::stride] += src in place (dauc_strided_add; the bits of torch's add_)."""
    _cl_bf16(dx, "dx")
    _cl_bf16(src, "src")
    N, C, H, W = dx.shape
    if tuple(src.shape) != (N, C, (H - 1) // stride + 1, (W - 1) // stride + 1) or src.device != dx.device:
        raise ValueError(f"src must be {[N, C, (H - 1) // stride + 1, (W - 1) // stride + 1]} on {dx.device}")
    check(_lib.load().dauc_strided_add(_ptr(dx), _lib.DTYPE_BF16, N, H, W, C, int(stride), _ptr(src),
                                       _stream(dx.device)), "dauc_strided_add")
    return dx


def broadcast_hw(g: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """g [N, C] (or [N, C, 1, 1]) broadcast to a channels-last [N, C, H, W] tensor (dauc_broadcast_hw)."""
    _require(g, "g", torch.bfloat16)
    N, C = g.shape[0], g.shape[1]
    g2 = g.reshape(N, C).contiguous()
    if C % 8 or g2.data_ptr() % 16:
        raise ValueError("g must have C % 8 == 0")
    out = torch.empty((N, C, H, W), dtype=g.dtype, device=g.device, memory_format=torch.channels_last)
    check(_lib.load().dauc_broadcast_hw(_ptr(g2), _lib.DTYPE_BF16, N, H * W, C, _ptr(out), _stream(g.device)),
          "dauc_broadcast_hw")
    return out


def set_wgrad_form(form: int) -> None:
    """The tuning build's 3x3 weight-gradient form (dauc_set_wgrad_form): 0 automatic, 1 gather, 2 / 3 window with 64- / 128-pixel chunks,
    4 / 5 the same with shared window rows."""
    check(_lib.tuning().dauc_set_wgrad_form(int(form)), "dauc_set_wgrad_form")


def probe_tr16() -> torch.Tensor:
    """The wgrad kernel's transposing-read lane map (tuning build): [64 lanes, 8] int16."""
    out = torch.zeros((64, 8), dtype=torch.int16, device="cuda")
    check(_lib.tuning().dauc_probe_tr16(_ptr(out), _stream(out.device)), "dauc_probe_tr16")
    return out


def set_direct_fault(mode: int) -> None:
    """Fault injection into the direct count-index build of the tuning build (dauc_set_direct_fault,
    include/dauc_tuning.h): 0 none, 1 / 2 / 3 a corrupted cell index or counter. Tests only."""
    check(_lib.tuning().dauc_set_direct_fault(int(mode)), "dauc_set_direct_fault")


def set_index_form(form: int) -> None:
    """The count index's build in the exact-AUC evaluations of the tuning build (dauc_set_index_form;
    the one-call and the two-step forms): 0 the product's cell-slotted build, 1 round 5's direct
    build (count, blocks, scatter). Same integers; for A/B measurements and tests. Set it before the
    compaction."""
    check(_lib.tuning().dauc_set_index_form(int(form)), "dauc_set_index_form")


def set_search_mode(mode: int) -> None:
    """Search structure of the sort method (dauc_set_search_mode): 0 automatic (the count index
    where the table fits it and is not skewed, else the distinct-key index where the table holds
    at most 14,000 distinct keys, else the LDS search tree), 1 the tree, 2 the distinct-key index
    wherever it holds the table. Same integers in every mode; for tests and measurements (tuning
    build)."""
    check(_lib.tuning().dauc_set_search_mode(int(mode)), "dauc_set_search_mode")


__all__ = [
    "GradSeg", "label_map_phat", "surrogate_fwdbwd", "class_sums", "alpha_from_sums", "pd_update",
    "pd_update_dense", "coda_finalize", "scale_div", "split_scores", "pair_count", "auc_counts_sorted",
    "surrogate_logits_fwdbwd", "class_sums_logits", "surrogate_status",
    "sort_keys", "auc_counts_sorted_labeled", "compact_positives", "mode_code", "workspaces", "set_search_mode",
    "set_direct_fault", "set_index_form", "conv3x3_wgrad", "conv3x3_wgrad_supported", "stem_conv_forward", "stem_conv_wgrad",
    "stem_conv_supported", "strided_pick", "strided_add_", "broadcast_hw",
    "auc_eval_enqueue",
    "auc_slot_bytes",
    "auc_eval_compact_part",
    "auc_eval_query_part",
    "auc_eval_query_part_sorted",
]
