"""Run the product CoDA loop on TinyNet with the fixture's data and compare to the reference trajectory.

Shared by the GPU test (real HIP kernels on cuda:0) and the CPU gloo test
(host orchestration with the kernels swapped for the oracle, see cpu_kernels.py).

Tolerances: parameters, a, b, alpha, loss agree within 1e-5 relative (plus an
absolute floor of 1e-7, the fp32 resolution of O(1e-2) values); class counts and
step counters are exact; p_hat is exact (same fp32 ratio); BatchNorm running
buffers (never averaged) within 1e-5.
"""
from __future__ import annotations

import json

import numpy as np
import torch

import tinynet

RTOL = 1e-5
ATOL = 1e-7


def close(got, ref, what, rtol=RTOL, atol=ATOL):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    bad = np.abs(got - ref) > rtol * np.abs(ref) + atol
    if bad.any():
        i = np.flatnonzero(bad.reshape(-1))[0]
        raise AssertionError(f"{what}: {bad.sum()} mismatches, first at {i}: got {got.reshape(-1)[i]!r} "
                             f"ref {ref.reshape(-1)[i]!r}")


def run_rank(fixture: dict, rank: int, world: int, device, group=None, head: str = "softmax", graph: bool = False,
             collective: bool | None = None, eager_update: bool = False):
    from distributedauc_amd.coda import CoDA

    cfg = json.loads(str(fixture["config"]))
    net = tinynet.TinyNet()
    net.load_state_dict({k[len("init_"):]: torch.from_numpy(v) for k, v in fixture.items()
                         if k.startswith("init_")})
    if head == "logits":  # fold the softmax into the surrogate kernel
        net.softmax = torch.nn.Identity()
    net = net.to(device)
    coda = CoDA(net, lr=cfg["lr"], gamma=cfg["gamma"], T0=cfg["T0"], I=cfg["I"], split_index=cfg["split_index"],
                world=world, rank=rank, group=group, device=device, head=head, collective=collective)
    coda.use_graph(graph, eager_update=eager_update)
    xs, ys = fixture[f"r{rank}_x"], fixture[f"r{rank}_y"]

    def batches():
        for k in range(len(xs)):
            yield torch.from_numpy(xs[k]).to(device), torch.from_numpy(ys[k]).to(device)

    rec = {k: [] for k in ("w", "abalpha", "counts", "p_hat", "loss", "bn", "t_total")}
    st = coda.state

    def flat_params():
        return np.concatenate([p.detach().cpu().numpy().reshape(-1) for p in net.parameters()])

    def on_step(c):
        rec["w"].append(flat_params())
        rec["abalpha"].append(st.abalpha.cpu().numpy().copy())
        g = st.gcounts.cpu().numpy()
        lc = st.lcounts.cpu().numpy()
        rec["counts"].append([g[0], g[1], lc[0], lc[1]])
        rec["p_hat"].append(st.p_hat.cpu().numpy()[0])
        rec["loss"].append(c.last_loss.item())
        rec["bn"].append(np.concatenate([net.bn.running_mean.cpu().numpy(), net.bn.running_var.cpu().numpy()]))
        rec["t_total"].append(c.t_total)

    coda.run(batches(), num_stages=cfg["numStages"], total_iter=cfg["total_iter"], on_step=on_step)
    return {k: np.asarray(v) for k, v in rec.items()}, coda


def compare(fixture: dict, rank: int, rec: dict):
    p = f"r{rank}_"
    assert np.array_equal(rec["t_total"], fixture[p + "t_total"])
    assert np.array_equal(rec["counts"], fixture[p + "counts"]), (rec["counts"], fixture[p + "counts"])
    assert np.array_equal(rec["p_hat"].astype(np.float32), fixture[p + "p_hat"].astype(np.float32))
    close(rec["loss"], fixture[p + "loss"], "loss")
    close(rec["abalpha"], fixture[p + "abalpha"], "a/b/alpha")
    close(rec["w"], fixture[p + "w"], "parameters")
    close(rec["bn"], fixture[p + "bn"], "bn running buffers")
