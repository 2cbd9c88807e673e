"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container only (needs /root/reference, which never travels
to the GPU box):   python tests/golden/make_golden.py

The reference (ZhishuaiGuo/DistributedAUC, imagenet/) is imported read-only
with a stub ``torchvision`` module (torchvision is not installed and is only
used inside main.train(), main.py:94-102). Its own functions produce the
outputs: main.dppd_sg, main.average_all (over gloo), main.AUC and
data_partitioner.DataPartitioner. The loss is an inline expression in the
reference (main.py:313-317), so it is evaluated through
oracle.reference_cpu.surrogate_loss, whose text is pinned to those lines.

Output (small .npz / .json data files, inputs and expected outputs only):
  surrogate_cases.npz  loss + gradients (torch fp32 autograd) and fp64 closed form
  dppd_sg.npz          main.dppd_sg on a small module
  auc_cases.npz        main.AUC + sklearn integer counts on tie-heavy cases
  partitions.json      sha256 of DataPartitioner index lists
  coda_w{1,2,4}.npz    per-rank trajectory of a 2-stage CoDA run on TinyNet
  coda_w8_I*.npz       8 ranks at I = 1 (2 stages), 8 and 32 (3 stages): BASELINE configs[2]'s periods
"""
from __future__ import annotations

import copy
import hashlib
import json
import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path(os.environ.get("DAUC_REFERENCE", "/root/reference/imagenet"))
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))

from oracle import reference_cpu as R  # noqa: E402
import tinynet  # noqa: E402


def import_reference():
    sys.argv = ["main.py"]
    tv = types.ModuleType("torchvision")
    tv.transforms = types.ModuleType("torchvision.transforms")
    tv.datasets = types.ModuleType("torchvision.datasets")
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tv.transforms)
    sys.path.insert(0, str(REF))
    import data_partitioner  # noqa: F401
    import main

    return main, sys.modules["data_partitioner"]


# ---------------------------------------------------------------- surrogate
def gen_surrogate():
    rng = np.random.default_rng(7)
    cases = []
    for B in (1, 32, 256, 4097):
        for ppos in (0.001, 0.1, 0.5):
            cases.append((B, ppos, "uniform"))
    cases += [(65536, 0.1, "uniform"), (256, 1.0, "all_pos"), (256, 0.0, "all_neg"), (512, 0.3, "h01"), (300, 0.2, "zero_label")]
    out = {}
    for ci, (B, ppos, kind) in enumerate(cases):
        h = rng.random(B, dtype=np.float32)
        y = np.where(rng.random(B) < ppos, 1, -1).astype(np.int64)
        if B == 1 and ppos < 0.5:
            y[:] = -1
        if kind == "h01":
            h = (rng.random(B) < 0.5).astype(np.float32)
        if kind == "zero_label":
            y[rng.random(B) < 0.1] = 0  # neither class (masks are exact == +/-1)
        a, b, al = (np.float32(v) for v in rng.normal(0, 0.3, 3))
        p = np.float32(max(min(ppos + rng.normal(0, 0.01), 0.999), 0.001))
        F, dh, da, db, dal = R.surrogate_fwdbwd_fp32(h, y, a, b, al, p)
        F64, dh64, da64, db64, dal64 = R.surrogate_closed_form(h, y, a, b, al, p)
        out[f"c{ci}_h"] = h
        out[f"c{ci}_y"] = y.astype(np.int8)
        out[f"c{ci}_abap"] = np.array([a, b, al, p], np.float32)
        out[f"c{ci}_fp32"] = np.array([F, da, db, dal], np.float32)
        out[f"c{ci}_dh32"] = dh.astype(np.float32)
        out[f"c{ci}_fp64"] = np.array([F64, da64, db64, dal64], np.float64)
    out["ncases"] = np.array(len(cases))
    np.savez_compressed(HERE / "surrogate_cases.npz", **out)


# ---------------------------------------------------------------- dppd_sg
def gen_dppd(main):
    torch.manual_seed(5)
    net = torch.nn.Sequential(torch.nn.Linear(40, 30), torch.nn.BatchNorm1d(30), torch.nn.Linear(30, 2))
    for p in net.parameters():
        p.grad = torch.randn_like(p) * 0.1
    model0 = {k: (v + 0.01 * torch.randn_like(v)) if v.is_floating_point() else v
              for k, v in copy.deepcopy(net.state_dict()).items()}
    mk = lambda v: torch.tensor([v], dtype=torch.float32, requires_grad=True)  # noqa: E731
    a, b, alpha = mk(0.2), mk(-0.1), mk(0.3)
    for t, g in ((a, 0.05), (b, -0.02), (alpha, 0.07)):
        t.grad = torch.tensor([g], dtype=torch.float32)
    a0, b0, alpha0 = (torch.tensor([v], dtype=torch.float32) for v in (0.15, -0.05, 0.25))
    names = [n for n, _ in net.named_parameters()]
    before = {n: p.detach().clone().numpy() for n, p in net.named_parameters()}
    grads = {n: p.grad.clone().numpy() for n, p in net.named_parameters()}
    lr, gamma = 0.1, 2000.0
    main.dppd_sg(net, a, b, alpha, model0, a0, b0, alpha0, lr, gamma)
    after = {n: p.detach().numpy() for n, p in net.named_parameters()}
    cat = lambda d: np.concatenate([d[n].reshape(-1) for n in names])  # noqa: E731
    np.savez_compressed(
        HERE / "dppd_sg.npz",
        w=cat(before), g=cat(grads), w0=np.concatenate([model0[n].numpy().reshape(-1) for n in names]),
        w_new=cat(after), lr=np.float64(lr), gamma=np.float64(gamma),
        scalars=np.array([0.2, -0.1, 0.3], np.float32), grad3=np.array([0.05, -0.02, 0.07], np.float32),
        anchor3=np.array([0.15, -0.05, 0.25], np.float32),
        scalars_new=np.array([a.item(), b.item(), alpha.item()], np.float32),
    )


# ---------------------------------------------------------------- AUC
def gen_auc(main):
    from sklearn.metrics._ranking import _binary_clf_curve

    rng = np.random.default_rng(11)
    cases = {}
    def add(name, y, s):
        cases[name] = (np.asarray(y, np.int64), np.asarray(s, np.float32))

    add("two", [1, -1], [0.7, 0.3])
    add("two_tie", [1, -1], [0.5, 0.5])
    add("signed_zero", [1, -1, 1, -1], [0.0, -0.0, -0.0, 0.0])
    add("single_pos", np.r_[1, -np.ones(999)], rng.random(1000))
    add("all_equal", np.where(rng.random(500) < 0.3, 1, -1), np.full(500, 0.25))
    add("subnormal", [1, -1, 1, -1, -1], [1e-45, 0.0, 2e-45, 1e-45, -1e-45])
    add("rand_1k", np.where(rng.random(1000) < 0.1, 1, -1), rng.random(1000))
    add("ties_1k", np.where(rng.random(1000) < 0.5, 1, -1), np.round(rng.random(1000) * 16) / 16)
    add("rand_64k", np.where(rng.random(65536) < 0.01, 1, -1), rng.random(65536))
    add("ties_64k", np.where(rng.random(65536) < 0.2, 1, -1), np.floor(rng.random(65536) * 4096) / 4096)
    add("neg_scores", np.where(rng.random(4000) < 0.3, 1, -1), rng.normal(0, 1e3, 4000))
    out = {}
    for name, (y, s) in cases.items():
        auc = main.AUC(torch.from_numpy(y), torch.from_numpy(s))
        fps, tps, _ = _binary_clf_curve(y, s, pos_label=1)
        fps0, tps0 = np.r_[0, fps], np.r_[0, tps]
        two_u = int(np.sum(np.diff(fps0).astype(object) * (tps0[1:] + tps0[:-1]).astype(object)))
        c = R.auc_counts(y, s)
        assert c["two_u"] == two_u, (name, c, two_u)
        out[f"{name}_y"] = y
        out[f"{name}_s"] = s
        out[f"{name}_auc"] = np.float64(auc)
        out[f"{name}_counts"] = np.array([c["wins"], c["ties"], c["P"], c["N"], two_u], np.int64)
    out["names"] = np.array(list(cases))
    np.savez_compressed(HERE / "auc_cases.npz", **out)


# ---------------------------------------------------------------- partitioner
def gen_partitions(dp):
    class FakeImageNet:
        def __len__(self):
            return 1281167

    res = {}
    for keep in (0.4, 1.0):
        for size in (1, 2, 4, 8, 16):
            sizes = [0.01] + [(1 - 0.01) / size for _ in range(size)]
            part = dp.DataPartitioner(FakeImageNet(), sizes, seed=123, neg_keep_ratio=keep)
            res[f"keep{keep}_size{size}"] = [
                {"len": len(p), "sha256": hashlib.sha256(np.asarray(p, np.int64).tobytes()).hexdigest(),
                 "head": [int(v) for v in p[:5]]}
                for p in part.partitions
            ]
    (HERE / "partitions.json").write_text(json.dumps(res, indent=1))


# ---------------------------------------------------------------- CoDA trajectory
def _coda_rank(rank, world, port, outdir, overrides=None, nbatches=32):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    main, _ = import_reference()
    main.size = world  # average_all reads the module-global `size` (main.py:52-54)
    cfg = dict(tinynet.CONFIG, **(overrides or {}))
    net = tinynet.TinyNet()
    net.load_state_dict(tinynet.initial_state())
    xs, ys = tinynet.make_batches(rank, nbatches)
    it = iter(range(nbatches))

    def next_batch():
        k = next(it)
        return torch.from_numpy(xs[k]).clone(), torch.from_numpy(ys[k]).clone()

    names = [n for n, _ in net.named_parameters()]
    flat = lambda: np.concatenate([p.detach().numpy().reshape(-1) for p in net.parameters()])  # noqa: E731
    bn_state = lambda: np.concatenate([net.bn.running_mean.numpy(), net.bn.running_var.numpy()])  # noqa: E731
    rec = {k: [] for k in ("w", "abalpha", "counts", "p_hat", "loss", "bn", "t_total")}
    stage_rec = {k: [] for k in ("w_start", "alpha", "sums", "w_avg_end")}

    a = torch.zeros(1, requires_grad=True)
    b = torch.zeros(1, requires_grad=True)
    alpha = torch.zeros(1, requires_grad=True)
    t_total = 0
    local_total_pos = torch.zeros(1)
    local_total_neg = torch.zeros(1)
    global_total_pos = torch.zeros(1)
    global_total_neg = torch.zeros(1)
    p_hat = torch.zeros(1)
    net.zero_grad()
    with torch.no_grad():
        main.average_all(net, a, b, alpha, global_total_pos, global_total_neg,
                         local_total_pos, local_total_neg, None)
    rec0 = flat()
    for s in np.arange(1, cfg["numStages"]):  # main.py:144
        if s > 1:  # main.py:148-152
            for name, param in net.named_parameters():
                param.data = net_average[name]
            a.data = a_average
            b.data = b_average
        net0 = copy.deepcopy(net.state_dict())  # main.py:154
        stage_rec["w_start"].append(flat())
        h_neg, N_neg, h_pos, N_pos = (torch.zeros(1) for _ in range(4))
        net.eval()
        with torch.no_grad():
            for _ in range(3 ** int(s)):  # main.py:172-188
                x, lab = next_batch()
                lab[lab <= cfg["split_index"]] = -1
                lab[lab > cfg["split_index"]] = 1
                h_neg += torch.sum(net(x)[:, 1] * (-1 == lab).float())
                N_neg += torch.sum(-1 == lab)
                h_pos += torch.sum(net(x)[:, 1] * (1 == lab).float())
                N_pos += torch.sum(1 == lab)
        net.train()
        for t_ in (h_neg, N_neg, h_pos, N_pos):
            dist.all_reduce(t_, op=dist.ReduceOp.SUM)
        alpha.data = h_neg / N_neg - h_pos / N_pos  # main.py:197
        stage_rec["alpha"].append(alpha.item())
        stage_rec["sums"].append([h_neg.item(), N_neg.item(), h_pos.item(), N_pos.item()])
        a0 = a.clone().detach()
        b0 = b.clone().detach()
        alpha0 = alpha.clone().detach()
        T = cfg["T0"] * (3 ** (int(s) - 1))
        lr = cfg["lr"] * ((1 / 3) ** (int(s) - 1))
        net_average = copy.deepcopy(net.state_dict())
        a_average = a0.clone().detach()
        b_average = b0.clone().detach()
        for t in range(T):  # main.py:210-336
            if t_total > cfg["total_iter"]:
                break
            x, lab = next_batch()
            t_total += 1
            if 0 == t_total % cfg["I"]:
                with torch.no_grad():
                    if world > 1:
                        main.average_all(net, a, b, alpha, global_total_pos, global_total_neg,
                                         local_total_pos, local_total_neg, None)
                    else:
                        global_total_neg += local_total_neg
                        global_total_pos += local_total_pos
                    local_total_neg = 0
                    local_total_pos = 0
            lab[lab <= cfg["split_index"]] = -1
            lab[lab > cfg["split_index"]] = 1
            local_total_pos += torch.sum(1 == lab)
            local_total_neg += torch.sum(-1 == lab)
            p_hat = p_hat * 0 + float(global_total_pos + local_total_pos) / \
                float(global_total_pos + local_total_pos + global_total_neg + local_total_neg)
            score = net(x)[:, 1]
            loss = R.surrogate_loss(score, lab, a, b, alpha, p_hat)
            net.zero_grad()
            try:
                a.grad.data *= 0
                b.grad.data *= 0
                alpha.grad *= 0
            except Exception:
                pass
            loss.backward(retain_graph=True)
            main.dppd_sg(net, a, b, alpha, net0, a0, b0, alpha0, lr, cfg["gamma"])
            for name, param in net.named_parameters():
                net_average[name] = net_average[name] + param.data
            rec["w"].append(flat())
            rec["abalpha"].append([a.item(), b.item(), alpha.item()])
            rec["counts"].append([float(global_total_pos), float(global_total_neg),
                                  float(local_total_pos), float(local_total_neg)])
            rec["p_hat"].append(p_hat.item())
            rec["loss"].append(loss.item())
            rec["bn"].append(bn_state())
            rec["t_total"].append(t_total)
        for name, param in net.named_parameters():
            net_average[name] = net_average[name] / T
        stage_rec["w_avg_end"].append(np.concatenate([net_average[n].numpy().reshape(-1) for n in names]))
    out = {k: np.asarray(v) for k, v in rec.items()}
    out.update({f"stage_{k}": np.asarray(v) for k, v in stage_rec.items()})
    out["w_init_avg"] = rec0
    out["x"] = xs
    out["y"] = ys
    np.savez_compressed(Path(outdir) / f"rank{rank}.npz", **out)
    dist.destroy_process_group()


def gen_coda(world, port, overrides=None, suffix="", nbatches=32):
    """coda_w{world}{suffix}.npz; overrides replace tinynet.CONFIG entries (e.g. the averaging
    period I and the stage count, for BASELINE configs[2]'s I sweep at 8 ranks)."""
    import tempfile

    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_coda_rank, args=(world, port, td, overrides, nbatches), nprocs=world, join=True)
        merged = {}
        for r in range(world):
            with np.load(Path(td) / f"rank{r}.npz") as z:
                for k in z.files:
                    merged[f"r{r}_{k}"] = z[k]
    init = tinynet.initial_state()
    for k, v in init.items():
        merged[f"init_{k}"] = v.numpy()
    merged["world"] = np.array(world)
    merged["config"] = np.array(json.dumps(dict(tinynet.CONFIG, **(overrides or {}))))
    np.savez_compressed(HERE / f"coda_w{world}{suffix}.npz", **merged)


# BASELINE configs[2] (8 ranks, I in {1, 8, 32}) on TinyNet: 4 stages = 3 + 9 + 27 = 39 steps, so
# I = 8 averages 4 times and I = 32 once; the stage-s alpha estimate reads 3^s batches per rank
CODA_W8 = (("_I1", dict(I=1), 32), ("_I8_s4", dict(I=8, numStages=4), 80), ("_I32_s4", dict(I=32, numStages=4), 80))


if __name__ == "__main__":
    import sys

    if sys.argv[1:] == ["coda8"]:  # only the 8-rank period fixtures
        import_reference()
        for i, (suffix, ov, nb) in enumerate(CODA_W8):
            gen_coda(8, 29620 + i, ov, suffix, nb)
        print("8-rank CoDA fixtures written to", HERE)
        sys.exit(0)
    main, dp = import_reference()
    gen_surrogate()
    gen_dppd(main)
    gen_auc(main)
    gen_partitions(dp)
    for w, port in ((1, 29611), (2, 29612), (4, 29614)):
        gen_coda(w, port)
    for i, (suffix, ov, nb) in enumerate(CODA_W8):
        gen_coda(8, 29620 + i, ov, suffix, nb)
    print("golden fixtures written to", HERE)
