"""Autograd entry of the fused min-max square-loss AUC surrogate.

Replaces the inline expression of main.py:313-317 and its autograd backward
(main.py:326). The HIP kernel produces F, dF/dh and the three scalar gradients
in the forward pass (one read of h and y); backward only hands the stored dF/dh
to the backbone. The gradients of (a, b, alpha) are written straight into the
caller's ``grad3`` buffer (the CoDA flat gradient tail), where the update kernel
reads them, so they never enter autograd.
"""
from __future__ import annotations

import torch

from . import ops

_UNIT: dict = {}  # device -> 0-dim fp32 tensor 1.0, never written (the backward seed of a training step)


def unit_seed(device: torch.device) -> torch.Tensor:
    """The gradient seed ``loss.backward(unit_seed(loss.device))`` passes instead of a fresh
    ``ones_like(loss)``: the surrogate's backward recognises it by its storage and hands its
    stored dF/dh on without the ``* grad_out`` pass (the same bits: x * 1.0 == x)."""
    t = _UNIT.get(device)
    if t is None:
        t = _UNIT[device] = torch.ones((), dtype=torch.float32, device=device)
    return t


def _is_unit(grad_out: torch.Tensor) -> bool:
    t = _UNIT.get(grad_out.device)
    return t is not None and grad_out.dim() == 0 and grad_out.data_ptr() == t.data_ptr()


class AUCSurrogate(torch.autograd.Function):
    """F(h; a, b, alpha, p) with dF/dh, dF/da, dF/db, dF/dalpha from one kernel pass."""

    @staticmethod
    def forward(ctx, h, y, abalpha, p_hat, grad3):
        dh = torch.empty(h.shape[0], dtype=torch.float32, device=h.device)
        loss = torch.empty((), dtype=torch.float32, device=h.device)
        g3 = grad3 if grad3 is not None else torch.empty(3, dtype=torch.float32, device=h.device)
        ops.surrogate_fwdbwd(h, y, abalpha, p_hat, dh=dh, grad3=g3, loss=loss)
        ctx.save_for_backward(dh, g3)
        ctx.abalpha_grad = abalpha.requires_grad
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        dh, g3 = ctx.saved_tensors
        unit = _is_unit(grad_out)
        d_ab = (g3 if unit else g3 * grad_out) if ctx.abalpha_grad else None
        return dh if unit else dh * grad_out, None, d_ab, None, None


def auc_surrogate(h: torch.Tensor, y: torch.Tensor, abalpha: torch.Tensor, p_hat: torch.Tensor,
                  grad3: torch.Tensor | None = None) -> torch.Tensor:
    """Loss of main.py:313-317 for scores ``h`` (1-D, any stride) and labels ``y`` (+1/-1).

    abalpha: fp32 [3] = (a, b, alpha); p_hat: fp32 [1]. If ``grad3`` is given, the
    kernel writes (dF/da, dF/db, dF/dalpha) into it during the forward pass.
    """
    return AUCSurrogate.apply(h, y, abalpha, p_hat, grad3)


class AUCSurrogateLogits(torch.autograd.Function):
    """The same loss from the [B, 2] logits with the softmax column fused.

    Backward hands dF/dz (same dtype as z) to the backbone: the softmax forward and
    backward kernels (resnet.py:159, 218) are not run at all.
    """

    @staticmethod
    def forward(ctx, z, y, abalpha, p_hat, grad3):
        dz = torch.empty_like(z, memory_format=torch.contiguous_format)
        loss = torch.empty((), dtype=torch.float32, device=z.device)
        g3 = grad3 if grad3 is not None else torch.empty(3, dtype=torch.float32, device=z.device)
        ops.surrogate_logits_fwdbwd(z, y, abalpha, p_hat, dz=dz, grad3=g3, loss=loss)
        ctx.save_for_backward(dz, g3)
        ctx.abalpha_grad = abalpha.requires_grad
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        dz, g3 = ctx.saved_tensors
        unit = _is_unit(grad_out)
        d_ab = (g3 if unit else g3 * grad_out) if ctx.abalpha_grad else None
        return dz if unit else dz * grad_out.to(dz.dtype), None, d_ab, None, None


def auc_surrogate_logits(z: torch.Tensor, y: torch.Tensor, abalpha: torch.Tensor, p_hat: torch.Tensor,
                         grad3: torch.Tensor | None = None) -> torch.Tensor:
    """Loss of main.py:313-317 from 2-way logits z [B, 2] (fp32 or bf16), h = softmax(z)[:, 1]."""
    if not z.is_contiguous():
        z = z.contiguous()
    return AUCSurrogateLogits.apply(z, y, abalpha, p_hat, grad3)
