"""BASELINE configs[1] and configs[0] at their real sizes on the GPU, through the bench's own setup.

configs[1]: ResNet-50 CoDA, batch 256, 224^2, bf16 autocast backbone -- the headline workload:
161 parameter tensors, 23,512,130 fp32 parameters, one pd_update launch over all of them.
configs[0]: ResNet-18 CoDA, batch 32, 224^2, averaging period I = 8.

For a few real steps (an averaging round included) each test checks:
  * the update launch bit-exact against the C oracle (oracle/auc_oracle.c, main.py:61 + 333-334)
    on the gradients autograd produced, for every one of the parameters, and the scalar
    update (main.py:58-59, 64) against the oracle's restatement;
  * the class counts exact (main.py:307-308, 49-50) against the labels actually drawn;
  * a finite loss, and the all-reduced payload size (parameters + a, b, alpha + 2 counts).
The backbone (PyTorch-ROCm convolutions plus the HIP BN / max-pool / weight-gradient / stem kernels,
each parity-tested on its own in tests/test_{fused_bn,maxpool,conv_wgrad,conv_stem,weight_shadow}_gpu.py)
is not compared to a CPU run as a whole: different conv kernels."""
from __future__ import annotations

import sys
from pathlib import Path

import pytest
import torch

import update_check

pytestmark = pytest.mark.gpu
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def _run(arch, batch, I, steps, expect_tensors, expect_params, dev):
    import bench

    coda, it = bench.make_coda(arch, batch, 224, I, 0.1, 2, 1, 0, dev)
    st = coda.state
    assert len(st.entries) == expect_tensors and st.numel() == expect_params
    assert st.n_reduce * 4 == (st.n_params + 5) * 4 and st.n_params >= expect_params
    checks = update_check.install(coda, arch)
    pos = neg = 0
    for _ in range(steps):
        x, labels = next(it)
        pos += int((labels > 499).sum())
        neg += int((labels <= 499).sum())
        loss = coda.train_step(x, labels)
        assert torch.isfinite(loss).item()
    torch.cuda.synchronize()
    assert checks["updates"] == steps
    # every label counted exactly once: rounds fold the locals into the global fp32 counters
    # (begin_stage's alpha-estimate batches are not counted, main.py:172-188)
    total = (st.gcounts + st.lcounts).cpu().numpy()
    assert total.tolist() == [float(pos), float(neg)], (total, pos, neg)
    assert coda.t_total == steps and steps >= I  # at least one averaging round ran inside
    return coda


@pytest.mark.timeout(600)
def test_configs1_resnet50_b256(dev):
    """configs[1]: 161 tensors, 23,512,130 parameters, one 161-segment update launch per step."""
    _run("resnet50", 256, 4, 5, 161, 23_512_130, dev)


@pytest.mark.timeout(600)
def test_configs0_resnet18_b32_I8(dev):
    """configs[0] on the GPU: ResNet-18 (62 tensors, 11,177,538 parameters), batch 32, I = 8."""
    _run("resnet18", 32, 8, 9, 62, 11_177_538, dev)
