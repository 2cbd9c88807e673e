"""Check every pd_update launch of a CoDA rank against the C oracle (test helper, not product).

install(coda) replaces coda.state.update with a wrapper that captures everything the launch reads
(w, w0, avg, the gradients autograd left, the scalars), runs the real launch, and compares the
result with oracle/auc_oracle.c's restatement of main.py:61 + 333-334 bit for bit over every
parameter, and the scalar update (main.py:58-59, 64) with oracle/reference_cpu.py's.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import coracle
from oracle import reference_cpu as R


def dense(t: torch.Tensor, like: torch.Tensor) -> np.ndarray:
    """t's elements in `like`'s physical order (the flat buffer's order)."""
    if t.stride() != like.stride():
        t = torch.empty_like(like).copy_(t)
    return torch.as_strided(t, (t.numel(),), (1,)).detach().cpu().numpy()


def install(coda, tag: str = "") -> dict:
    st = coda.state
    checks = {"updates": 0}
    orig_update = st.update

    def gather(buf):
        return np.concatenate([buf[o:o + n].cpu().numpy() for _, _, o, n in st.entries])

    def checked_update(lr, gamma, mode="reference", running_average=True):
        torch.cuda.synchronize()
        w, w0, avg = gather(st.flat), gather(st.anchor), gather(st.avg)
        g = np.concatenate([dense(p.grad, p) for _, p, _, _ in st.entries])
        sc, g3, an = st.abalpha.cpu().numpy(), st.grad3.cpu().numpy(), st.anchor3.cpu().numpy()
        orig_update(lr, gamma, mode, running_average)
        torch.cuda.synchronize()
        ew, eavg = coracle.pd_update(w, g, w0, lr, gamma, avg)
        assert np.array_equal(gather(st.flat), ew), f"{tag}: parameters differ from the oracle at step {coda.t_total}"
        assert np.array_equal(gather(st.avg), eavg), f"{tag}: running average differs at step {coda.t_total}"
        ea, eb, eal = R.scalar_update(*sc[:3], *g3[:3], *an[:3], lr, gamma, mode)
        assert st.abalpha.cpu().numpy().tolist() == [ea, eb, eal], f"{tag}: a, b, alpha at step {coda.t_total}"
        checks["updates"] += 1

    st.update = checked_update
    return checks
