"""The reference-side ctypes binding shown in INTEGRATION.md §2, executed verbatim against libdauc.so:
its AUC() (the one blocking call dauc_auc_eval_counts) must give the C oracle's exact counts, and
its dppd_sg_param() the oracle's bit-exact update (main.py:61)."""
from __future__ import annotations

import re
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import coracle

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _stub():
    text = (REPO / "INTEGRATION.md").read_text()
    sec = text[text.index("## 2. Bind the C ABI directly"):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    code = code.replace('ctypes.CDLL("libdauc.so")', f'ctypes.CDLL("{REPO / "distributedauc_amd" / "libdauc.so"}")')
    ns: dict = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    return ns


def test_integration_stub_auc_and_update(dev):
    ns = _stub()
    rng = np.random.default_rng(11)
    for n, p, q in ((1000, 0.1, 0), (300_007, 0.01, 1024), (300_007, 0.9, 1024), (2_000_000, 0.002, 0)):
        s = rng.random(n, dtype=np.float32)
        if q:
            s = (np.floor(s * q) / q).astype(np.float32)
        y = np.where(rng.random(n) < p, 1, -1).astype(np.int8)
        e = coracle.auc_counts(y.astype(np.int64), s)
        got = ns["AUC"](torch.from_numpy(y), torch.from_numpy(s))
        assert got == (2 * e["wins"] + e["ties"]) / (2 * e["P"] * e["N"])
    y[5], s[5] = -1, np.nan  # a non-finite negative: only the query pass sees it
    with pytest.raises(ValueError):
        ns["AUC"](torch.from_numpy(y), torch.from_numpy(s))
    w, g, w0 = (rng.standard_normal(4099).astype(np.float32) for _ in range(3))
    tw = torch.from_numpy(w).to(dev)
    tw.grad = torch.from_numpy(g).to(dev)
    ns["dppd_sg_param"](tw, torch.from_numpy(w0).to(dev), 0.1, 2000.0)
    torch.cuda.synchronize()
    assert np.array_equal(tw.cpu().numpy(), coracle.pd_update(w, g, w0, 0.1, 2000.0))
