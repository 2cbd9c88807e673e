"""Flat HBM layout of one CoDA rank's state.

The reference keeps 161 separate parameter tensors (ResNet-50) plus scalar
tensors a, b, alpha and four count tensors, and touches each of them with
several small kernels per step (main.py:56-64, 124-133, 333-334). Here every
trainable parameter of the backbone is a view into ONE contiguous fp32 buffer,
followed by the AUC scalars and the per-round class counts:

    flat  = [ p_0 | pad | p_1 | pad | ... | p_last | pad | a b alpha | lpos lneg | pad ]
             \------------- n_params (multiple of 64) -------------/ \- n_avg-/ \ n_reduce /

    anchor = same first n_avg elements : (w0, a0, b0, alpha0)   main.py:154-158, 199-201
    avg    = first n_params elements   : running average        main.py:206, 333-334

so that:
  * a CoDA round is ONE all-reduce of flat[:n_reduce] (parameters, a, b, alpha
    and the local class counts, which are exact small integers in fp32) and ONE
    finalise kernel (divide by world, fold counts);
  * the primal-dual update + running average is ONE bandwidth-bound kernel over
    flat/anchor/avg, reading each parameter's gradient where autograd left it.

BatchNorm running buffers are NOT in the flat buffer: the reference does not
average them (main.py:35 iterates model.parameters() only).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from ._lib import GradSeg

ALIGN = 64  # elements: every parameter view starts on a 256-byte boundary
TAIL = 8    # a, b, alpha, lpos, lneg + 3 pad (keeps the buffer a multiple of 16 B)


def _check_device(dev: torch.device) -> None:
    if dev.type != "cuda":
        raise RuntimeError(f"FlatState lives in GPU memory; got device {dev}")


def _dense_layout(t: torch.Tensor) -> bool:
    """True if t's elements occupy exactly numel contiguous slots (any dim order)."""
    if t.numel() <= 1:
        return True
    dims = sorted((s, n) for s, n in zip(t.stride(), t.shape) if n != 1)
    expect = 1
    for s, n in dims:
        if s != expect:
            return False
        expect *= n
    return True


def _same_order(g: torch.Tensor, p: torch.Tensor) -> bool:
    """g's elements sit where p's do: equal strides on every dimension longer than 1 (a 1x1 conv
    weight's gradient [Cout, Cin, 1, 1] is the same memory whether its unit dimensions carry
    contiguous or channels-last strides -- autograd's layout contract ignores them too)."""
    if g.shape != p.shape or not _dense_layout(g):
        return False
    return all(n == 1 or gs == ps for n, gs, ps in zip(p.shape, g.stride(), p.stride()))


class FlatState:
    """One rank's CoDA state in four device buffers (see module docstring)."""

    def __init__(self, model: nn.Module, device: torch.device | str | None = None):
        params = [(n, p) for n, p in model.named_parameters()]
        if not params:
            raise ValueError("model has no parameters")
        dev = torch.device(device) if device is not None else params[0][1].device
        _check_device(dev)
        self.device = dev
        entries = []
        off = 0
        for name, p in params:
            if p.dtype != torch.float32:
                raise TypeError(f"parameter {name} is {p.dtype}; CoDA keeps fp32 master weights")
            if not _dense_layout(p):
                raise ValueError(f"parameter {name} is not densely laid out (strides {p.stride()})")
            entries.append((name, p, off, p.numel()))
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.n_params = off
        self.n_avg = off + 3       # parameters + a, b, alpha: divided by world
        self.n_reduce = off + 5    # + lpos, lneg: summed by the all-reduce
        self.flat = torch.zeros(off + TAIL, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for name, p, o, n in entries:
                view = torch.as_strided(self.flat, p.shape, p.stride(), o)
                view.copy_(p.detach().to(dev))
                p.data = view
        self.entries = entries
        self.params = self.flat[:off]
        self.abalpha = self.flat[off:off + 3]
        self.a = self.flat[off:off + 1]
        self.b = self.flat[off + 1:off + 2]
        self.alpha = self.flat[off + 2:off + 3]
        self.lcounts = self.flat[off + 3:off + 5]          # main.py:129-130 (lpos, lneg)
        self.anchor = torch.zeros(off + TAIL, dtype=torch.float32, device=dev)
        self.anchor3 = self.anchor[off:off + 3]             # a0, b0, alpha0
        self.avg = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad3 = torch.zeros(4, dtype=torch.float32, device=dev)   # dF/da, dF/db, dF/dalpha
        self.gcounts = torch.zeros(2, dtype=torch.float32, device=dev)  # main.py:131-132 (gpos, gneg)
        self.p_hat = torch.zeros(1, dtype=torch.float32, device=dev)    # main.py:133
        self._segs = (GradSeg * len(entries))()
        self._y8: dict[int, torch.Tensor] = {}
        model._dauc_flat = self

    # ------------------------------------------------------------------ helpers
    def y8(self, B: int) -> torch.Tensor:
        """Reusable int8 label buffer for a batch of B."""
        t = self._y8.get(B)
        if t is None:
            t = torch.empty(B, dtype=torch.int8, device=self.device)
            self._y8[B] = t
        return t

    def grad_segments(self):
        """Fill the segment table with every parameter's gradient pointer (host only)."""
        keep = []
        for i, (name, p, off, n) in enumerate(self.entries):
            g = p.grad
            if g is None:
                raise RuntimeError(f"parameter {name} has no gradient; run backward first")
            if g.dtype != torch.float32 or g.device != self.device:
                raise TypeError(f"gradient of {name} must be fp32 on {self.device}")
            if n > 1 and not _same_order(g, p):
                g = torch.empty_like(p).copy_(g)  # same physical order as the parameter
                keep.append(g)
            seg = self._segs[i]
            seg.grad = g.data_ptr()
            seg.offset = off
            seg.numel = n
        return self._segs, keep

    # ------------------------------------------------------------------ hot path
    def update(self, lr: float, gamma: float, mode: str = "reference", running_average: bool = True):
        """dppd_sg (main.py:56-64) + running average (main.py:333-334): one launch."""
        segs, keep = self.grad_segments()
        ops.pd_update(self.flat, self.anchor, self.avg if running_average else None, segs, len(self.entries),
                      scalars=self.abalpha, grad3=self.grad3, anchor3=self.anchor3, lr=lr, gamma=gamma,
                      mode=mode)
        del keep  # stream-ordered: the caching allocator reuses these only after the kernel

    def snapshot_anchor(self):
        """net0 / a0 / b0 / alpha0 <- current values (main.py:154-158, 199-201)."""
        self.anchor[: self.n_avg].copy_(self.flat[: self.n_avg])

    def reset_average(self):
        """net_average <- deepcopy(net.state_dict()) (main.py:206) for the parameters."""
        self.avg.copy_(self.params)

    def bytes_per_update(self, running_average: bool = True) -> int:
        """Algorithmic HBM bytes of one update launch: 16 B/param, 24 B with the average."""
        n = sum(e[3] for e in self.entries)
        return n * (24 if running_average else 16)

    def numel(self) -> int:
        return sum(e[3] for e in self.entries)
