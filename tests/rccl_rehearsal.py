"""The RCCL rehearsal: every collective the N > 1 path issues, on a one-rank
``nccl`` process group (= RCCL) on the one GPU the test box has, with the product's world > 1
branches forced on (``collective=True``). Run as the ONLY rank of ``torch.distributed.run
--nproc-per-node 1`` (a fresh process: the communicator is created before any other GPU work, as in
the driver's 8-GPU run). Writes one JSON record of what ran and what it gave to argv[1]; the GPU
test (tests/test_rccl_rehearsal_gpu.py) asserts on it. Reference: main.py:292-301 (averaging every
I steps), 33-54 (average_all), 192-195 (alpha all-reduce), 232-250 (evaluation), node0.sh:2-5
(the NCCL launch). TEST INFRASTRUCTURE: the oracle is the checker here, never the thing measured."""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
from distributedauc_amd import use_tuned_miopen_db  # noqa: E402

use_tuned_miopen_db()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def log(msg):
    print(f"[rehearsal {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main(out_path: str) -> None:
    if "WORLD_SIZE" not in os.environ:
        raise SystemExit("run under torch.distributed.run --nproc-per-node 1")
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)  # the communicator exists before any other GPU work
    world, rank = dist.get_world_size(), dist.get_rank()
    rec = {"backend": dist.get_backend(), "world": world, "rank": rank,
           "rccl_version": ".".join(map(str, torch.cuda.nccl.version())), "steps": []}

    def done(name, **kw):
        rec["steps"].append(dict(kw, step=name))
        log(f"{name}: {kw}")

    # 1. CoDA on the bench's ResNet-50 b256 bf16 (configs[1]): make_coda runs the pre-training
    #    averaging round (the 94 MB flat all-reduce + finalise, main.py:141-142) and the stage's
    #    alpha estimate (the fp64 [4] all-reduce, main.py:192-195) on the nccl group
    import bench
    from distributedauc_amd.coda import CoDA

    coda, it = bench.make_coda("resnet50", 256, 224, 16, 0.1, 2, world, rank, dev, lr=0.01)
    assert coda.collective and isinstance(coda, CoDA)
    st = coda.state
    x, y = next(it)
    coda.train_step(x, y)  # one step so the local counts are nonzero
    before = st.flat.clone()
    lc, gc = st.lcounts.clone(), st.gcounts.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    coda.average_all()  # all_reduce(flat[:n_reduce]) over RCCL + dauc_coda_finalize
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    done("coda_round_r50", payload_bytes=st.n_reduce * 4, n_reduce=st.n_reduce, seconds=dt,
         params_equal=bool(torch.equal(st.flat[: st.n_avg], before[: st.n_avg])),
         counts_folded=bool(torch.equal(st.gcounts, gc + lc)) and bool((st.lcounts == 0).all()),
         alpha=float(st.alpha.item()), alpha_finite=bool(torch.isfinite(st.alpha).all()))
    # training steps with averaging rounds inside them (I = 2: a round every second step)
    coda.I = 2
    losses = []
    for _ in range(4):
        x, y = next(it)
        losses.append(float(coda.train_step(x, y).item()))
    done("train_steps_r50_I2", losses=losses, finite=bool(np.isfinite(losses).all()))
    sums = torch.tensor([3.5, 7.0, -1.25, 2.0], dtype=torch.float64, device=dev)
    ref = sums.clone()
    dist.all_reduce(sums)
    done("alpha_sums_fp64", equal=bool(torch.equal(sums, ref)))
    del coda, it, before
    torch.cuda.empty_cache()

    # 2. the two-step sharded exact AUC at configs[3] and configs[4] sizes: the uint8 slot
    #    all_gather_into_tensor and the int64 record all-gather on RCCL; counts vs the C oracle
    from distributedauc_amd.auc import ExactAUC
    from distributedauc_amd.loader import synthetic_scores
    from oracle import coracle

    for log2n, pos in ((24, 0.01), (27, 0.001)):
        s, y = synthetic_scores(1 << log2n, pos, dev)
        ev = ExactAUC(world=world, rank=rank, collective=True, shard_min=0)
        c = ev.counts(y, s)
        mode = ev.last_mode
        e = coracle.auc_counts(y.cpu().numpy().astype(np.int64), s.cpu().numpy())
        done(f"auc_two_step_2^{log2n}", mode=mode, counts=c,
             match=(c["wins"], c["ties"], c["P"], c["N"]) == (e["wins"], e["ties"], e["P"], e["N"]))
        # the pair-count method's 6-word record all-gather
        if log2n == 24:
            cp = ExactAUC(world=world, rank=rank, collective=True, method="pairs").counts(y, s)
            done("auc_pairs_2^24", match=(cp["wins"], cp["ties"]) == (e["wins"], e["ties"]))
        del s, y
    torch.cuda.empty_cache()

    # 3. the split in-training evaluation: broadcast of rank 0's parameters and BN statistics,
    #    all-gather of the scores, sharded count (main.py:215-250)
    from distributedauc_amd.loader import DeviceLoader, SyntheticImageNet, imagenet_like_labels
    from distributedauc_amd.main import Evaluator

    coda, it = bench.make_coda("resnet18", 32, 64, 8, 0.1, 2, world, rank, dev)
    labels = imagenet_like_labels(512, 1000, 499, pos_ratio=0.1, seed=777)
    ds = SyntheticImageNet(labels, 64, 499)
    tit = iter(DeviceLoader(ds, np.arange(512), 64, dev, seed=777, shuffle=False, channels_last=True))
    batches = [next(tit) for _ in range(8)]
    ev = Evaluator(batches, 512, 499, dev, None, world, rank, None, split=True, collective=True)
    a = ev(coda)
    done("split_evaluation", split=ev.split_scoring, auc=a, finite=bool(np.isfinite(a)))
    del coda, it
    dist.barrier()
    done("barrier")

    # 4. HIP-graph capture of step_body AFTER the communicator exists, averaging rounds (RCCL,
    #    eager) between replays: the fixture's 2-stage trajectory (tests/golden/coda_w1.npz), graph
    #    vs eager bit for bit and both against the reference's trajectory
    import coda_parity

    fx = dict(np.load(REPO / "tests" / "golden" / "coda_w1.npz"))
    eager, _ = coda_parity.run_rank(fx, 0, 1, dev, collective=True)
    graphed, cg = coda_parity.run_rank(fx, 0, 1, dev, collective=True, graph=True)
    same = all(np.array_equal(eager[k], graphed[k]) for k in eager)
    ok_ref = True
    try:
        coda_parity.compare(fx, 0, graphed)
    except AssertionError as err:  # recorded, asserted by the test
        ok_ref = str(err)
    done("graph_after_comm", captures=cg.graph_captures, graph_equals_eager=same, matches_reference=ok_ref)

    dist.barrier()
    dist.destroy_process_group()
    Path(out_path).write_text(json.dumps(rec, default=str))
    log("done")


if __name__ == "__main__":
    main(sys.argv[1])
