"""Benchmark of the CoDA hot path on MI355X (driver contract: one JSON line from rank 0).

Headline (BASELINE.json configs[1]): ResNet-50 CoDA, bf16 autocast backbone,
batch 256 per GPU, 224x224 synthetic inputs already resident in HBM, p=0.1,
fused AUC surrogate + primal-dual update kernels, CoDA averaging every I=16
steps over RCCL. A step = label map/p_hat + forward + fused loss + backward +
update (+ the averaging round when t % I == 0). value = images/s of the whole
job (all ranks), timed over exactly --steps steps between barriers.

Other BASELINE configs, as sub-records of the same line:
  configs[2]  the averaging-period sweep I in {1, 8, 16, 32} of the same step (``period_sweep``)
              and one timed CoDA round (``coda_round``: the RCCL all-reduce + finalise, xGMI share)
  configs[0]  ResNet-18 b32 224^2 I=8 on the GPUs (``configs0.gpu``) next to the reference CPU
              path on 4 gloo worker processes (``configs0.cpu``: restated step + average_all)
  configs[3]  exact AUC of 2^24 scores at 1 % positives (``auc_eval``)
  configs[4]  exact AUC of 2^27 scores at 0.1 % positives (``auc_eval_extreme``), with the C
              oracle's counts on the full vector in its cpu_baseline
plus the loss kernel at a streaming size (``surrogate_kernel``).

Launch: ``python bench.py --gpus N`` with no launcher starts N rank processes itself (a
torch.distributed.run child, before this process touches the GPU) and exits with its code;
under a launcher (WORLD_SIZE set) it runs as one rank. The run fails if the process group's
size differs from --gpus.

Kernel timing: HIP events recorded on the stream each kernel is launched on
(torch's current stream, which is the stream libdauc.so receives), around every
launch inside the timed region. roofline.achieved = algorithmic bytes per launch
/ average launch duration.

    python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
from distributedauc_amd import use_tuned_miopen_db  # noqa: E402

use_tuned_miopen_db()  # before any convolution: the shipped MI355X find/perf db

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_BF16_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF bf16 dense MFMA (no sparsity)
# VALU ceilings of the pair count (pairs/s per GPU). Vector fp32 rate = 256 CU x 4 SIMD x 32
# lanes x 2.4 GHz = 7.86e13 lane-ops/s (157.3 TF / 2).
#   packed: the cheapest exact sequence on gfx950, 3 fp32 lane-ops per pair (v_pk_add_f32,
#           v_pk_fma_f32 clamp, v_pk_add_f32 over 2 pairs) -> 2.62e13
#   survey: SURVEY §8(d)'s bar, 2 compares per pair on 16-wide SIMDs -> 1.97e13
VALU_PAIR_PEAK = 2.62e13
SURVEY_PAIR_PEAK = 1.97e13
XGMI_PEAK_GBS = 7 * 153.0   # one GPU's 7 xGMI links x ~153 GB/s (the ring all-reduce's bus-bandwidth ceiling)
METRIC = "CoDA train imgs/sec + exact-AUC pos×neg pairs/sec at 1/2/4/8 MI355X"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--arch", default="resnet50")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--I", type=int, default=16)
    p.add_argument("--pos-ratio", type=float, default=0.1)
    p.add_argument("--lr", type=float, default=0.01,
                   help="CoDA step size. The reference runs lr 0.1 on a PRETRAINED ResNet-50 (node0.sh); from "
                        "random init at 0.1 its own loop saturates the softmax column within 5 steps (the CPU "
                        "oracle loop too: profiles/r04/direction/), so the in-training AUC is meaningless there. "
                        "0.01 learns the synthetic signal. The step's kernels and bytes do not depend on lr")
    p.add_argument("--pool", type=int, default=4, help="distinct resident input batches cycled")
    p.add_argument("--signal-flip", type=float, default=0.2,
                   help="fraction of the synthetic images (training and test) carrying the other class's sign "
                        "(loader.py): the best achievable test AUC is 1 - flip, so the in-training AUC can land "
                        "between chance and that ceiling instead of saturating at 1.0 (VERDICT r04 #7); shapes "
                        "and bytes of every step are unchanged")
    p.add_argument("--sweep-I", default="1,8,16,32", help="configs[2] averaging periods ('' = off)")
    p.add_argument("--sweep-steps", type=int, default=32, help="timed steps per period (a multiple of every I)")
    p.add_argument("--eval-images", type=int, default=8192,
                   help="in-training evaluation leg: test images scored with rank 0's model (0 = off)")
    p.add_argument("--r18-steps", type=int, default=16, help="configs[0] GPU leg: timed ResNet-18 b32 steps (0 = off)")
    p.add_argument("--r18-graph", type=int, default=1,
                   help="configs[0] GPU leg at N=1: replay the step body as a HIP graph (1/0); N>1 runs eager "
                        "(2 gloo ranks sharing one GPU replayed slower than eager: profiles/r02/graph/)")
    p.add_argument("--auc-log2n", type=int, default=24)
    p.add_argument("--auc-pos", type=float, default=0.01)
    p.add_argument("--auc-reps", type=int, default=3)
    p.add_argument("--auc-shard-min", type=int, default=None,
                   help="scores below which N > 1 ranks evaluate the whole vector instead of sharding "
                        "(default ExactAUC.SHARD_MIN = 2^24; 0 shards every size, for rehearsals)")
    p.add_argument("--auc2-log2n", type=int, default=27, help="configs[4] leg (0 = off)")
    p.add_argument("--auc2-pos", type=float, default=0.001)
    p.add_argument("--sur-log2b", type=int, default=26, help="surrogate kernel leg: batch of 2^k scores")
    p.add_argument("--sur-reps", type=int, default=100)
    p.add_argument("--variant", type=int, default=0, help="pair-count kernel variant")
    p.add_argument("--backend", default=None,
                   help="torch.distributed backend: nccl (= RCCL; the default at --gpus > 1) or gloo (shared-GPU "
                        "rehearsals). Given at --gpus 1, a one-rank process group of that backend is started through "
                        "torch.distributed.run and every collective of the N > 1 path runs on it (the RCCL rehearsal)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-baseline-any-n", action="store_true",
                   help="also time the CPU baselines when N > 1 (the contract times them at N = 1 only: rank 0's "
                        "CPU minutes would hold every other rank at the closing barrier)")
    p.add_argument("--cpu-workers", type=int, default=4, help="configs[0] CPU leg: gloo worker processes")
    p.add_argument("--cpu-steps", type=int, default=8, help="configs[0] CPU leg: timed steps (one round at I=8)")
    p.add_argument("--cpu-max-s", type=float, default=90.0,
                   help="all-core CPU baseline of configs[1]: skipped when its warm-up projects a longer timed step")
    p.add_argument("--cpu-sklearn-full", type=int, default=1,
                   help="time sklearn on the full configs[4] vector (1) or its first 2^24 scores (0)")
    p.add_argument("--no-auc", action="store_true")
    p.add_argument("--no-train", action="store_true")
    p.add_argument("--no-surrogate", action="store_true")
    p.add_argument("--fused-bn", type=int, default=1, help="fused BN+add+ReLU HIP kernels in the backbone (1/0)")
    p.add_argument("--graph", type=int, default=0,
                   help="headline step: replay label map -> forward -> surrogate -> backward from one HIP graph, "
                        "the update launched eagerly after each replay (1) or everything eager (0)")
    p.add_argument("--weight-shadow", type=int, default=3,
                   help="bf16 conv weights from one shadow cast per forward (1), + the stride-1 3x3 input "
                        "gradients as forward convolutions with flipped weights (2), + the 3x3 weight gradients "
                        "from the HIP MFMA kernel (3), or autocast's cast per conv (0)")
    p.add_argument("--bn-steps", type=int, default=3,
                   help="last warm-up steps with HIP events around every fused BN call (step_roofline.bn; 0 = off)")
    p.add_argument("--gemm-conv1x1", type=int, default=1,
                   help="stride-1 1x1 convs as hipBLASLt GEMMs where faster (per-shape timing; 1/0)")
    # internal: one process of the configs[0] CPU baseline (never touches the GPU)
    p.add_argument("--cpu-coda-worker", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--cpu-train-worker", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--cw-rank", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--cw-port", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--cw-threads", type=int, default=1, help=argparse.SUPPRESS)
    p.add_argument("--cw-out", default="", help=argparse.SUPPRESS)
    return p.parse_args(argv)


_last_log = ["start", time.time()]


def log(msg: str):
    _last_log[:] = [msg, time.time()]
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def start_heartbeat(period: float = 45.0) -> None:
    """A line on stderr whenever `period` seconds pass without one (long CPU-baseline legs, first
    MIOpen searches): a watchdog that reads silence as a hang sees the run alive."""
    import threading

    def beat():
        while True:
            time.sleep(period / 3)
            msg, t = _last_log
            if time.time() - t >= period:
                print(f"[bench {time.strftime('%H:%M:%S')}] still running: {msg} (+{time.time() - t:.0f} s)",
                      file=sys.stderr, flush=True)
                _last_log[1] = time.time()

    threading.Thread(target=beat, daemon=True).start()


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def host_info() -> dict:
    """The host CPU share this run may use (north_star: the core count must be stated)."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp == "1" and int(os.environ.get("LOCAL_WORLD_SIZE", "1")) > 1:
        # torch.distributed.run exports OMP_NUM_THREADS=1 when the environment had none; the CPU
        # baselines run on rank 0 alone while the other ranks wait, so use the default share
        omp = None
    budget = min(affinity, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else min(affinity, 16)
    quota = cgroup_cpus()
    usable = min(affinity, int(quota)) if quota else affinity  # CPUs of time the process can get
    return {"nproc": os.cpu_count(), "affinity_cpus": affinity, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "cpu_budget": budget, "cgroup_cpu_quota": quota, "usable_cpus": max(usable, 1)}


def cgroup_cpus():
    """The cgroup CPU quota in CPUs (cpu.max / cfs_quota_us), or None when unlimited / unreadable."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        return None if q < 0 else q / per
    except (OSError, ValueError):
        return None


# ----------------------------------------------------------------------------- timing helpers
class KernelTimer:
    """HIP events on the launch stream around every call of one libdauc.so entry point.

    The wrapper replaces the ctypes function on the loaded library, so only the C call
    (host launch + the kernel) sits between the two event records. The stream argument
    is the last parameter of every dauc_* entry point.
    """

    def __init__(self, lib, name, nbytes=None):
        self.lib, self.name = lib, name
        self.fn = getattr(lib, name)
        self.pairs = []
        self.bytes = 0  # algorithmic bytes of the timed calls (nbytes(args) per call), when given
        self.enabled = False
        fn = self.fn

        def wrapped(*a):
            if not self.enabled:
                return fn(*a)
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            r = fn(*a)
            e1.record(s)
            self.pairs.append((e0, e1))
            if nbytes is not None:
                self.bytes += nbytes(a)
            return r

        setattr(lib, name, wrapped)

    def restore(self):
        setattr(self.lib, self.name, self.fn)

    def mean_ms(self):
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b) for a, b in self.pairs])) if self.pairs else float("nan")

    def total_ms(self):
        torch.cuda.synchronize()
        return float(np.sum([a.elapsed_time(b) for a, b in self.pairs]))


# ----------------------------------------------------------------------------- step roofline
def _ival(v):
    return int(getattr(v, "value", v) or 0)


def _esize(dtype_code):
    return 2 if _ival(dtype_code) == 2 else 4  # DAUC_DTYPE_BF16 = 2, DAUC_DTYPE_F32 = 1


def bn_forward_bytes(a):
    """Algorithmic HBM bytes of one dauc_bn_act_forward call (csrc/bn_act.hip's two passes): the
    stats pass reads x; the apply pass reads x (+ residual) and writes y (+ the 1-bit ReLU mask, one
    byte per 16-byte vector). Per-channel vectors are negligible. Args: include/dauc.h order."""
    e, M, C = _esize(a[1]), _ival(a[2]), _ival(a[3])
    act = M * C * e
    residual, mask = _ival(a[4]) != 0, _ival(a[13]) != 0
    return act + act + (act if residual else 0) + act + (act // 16 if mask else 0)


def bn_backward_bytes(a):
    """One dauc_bn_act_backward call: the reduce pass reads dy, the ReLU mask (or y) and x (and writes
    dz = the residual's gradient when there is one); the dx pass reads dy + mask (or dz) and x and
    writes dx."""
    e, M, C = _esize(a[4]), _ival(a[5]), _ival(a[6])
    act = M * C * e
    relu, has_mask, has_y, dres = _ival(a[7]) != 0, _ival(a[2]) != 0, _ival(a[1]) != 0, _ival(a[11]) != 0
    g_src = (act // 16 if has_mask else act if has_y else 0) if relu else 0  # what the ReLU mask costs
    reduce = act + g_src + act + (act if dres else 0)
    dx = (act if dres else act + g_src) + act + act
    return reduce + dx


def backbone_flops(arch: str, image_size: int, batch: int) -> dict:
    """FLOP of one training step's convolutions and fc from the layer shapes (a forward on the meta
    device with hooks): forward 2 MAC, weight gradient 2 MAC, input gradient 2 MAC except for the
    stem (its input, the image, needs none). BN, pooling and the AUC kernels are not counted (they
    are bandwidth work: bn_roofline / the update and loss kernels' rooflines)."""
    from distributedauc_amd.backbone import build_backbone

    with torch.device("meta"):
        net = build_backbone(arch, num_classes=2)
    macs = []

    def hook(m, inp, out):
        if isinstance(m, torch.nn.Conv2d):
            kh, kw = m.kernel_size
            macs.append((m is net.conv1, out.numel() * (m.in_channels // m.groups) * kh * kw))
        elif isinstance(m, torch.nn.Linear):
            macs.append((False, out.numel() * m.in_features))

    hs = [m.register_forward_hook(hook) for m in net.modules() if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear))]
    with torch.no_grad():
        net(torch.empty((batch, 3, image_size, image_size), device="meta"))
    for h in hs:
        h.remove()
    fwd = sum(m for _, m in macs)
    stem = sum(m for first, m in macs if first)
    flop = 2 * fwd + 2 * fwd + 2 * (fwd - stem)
    return {"forward_gmac": fwd / 1e9, "flop_per_step": flop, "layers": len(macs)}


def grouped() -> bool:
    """A process group is up: the N > 1 path (and its collectives) runs, at any world size."""
    return dist.is_available() and dist.is_initialized()


def max_over_ranks(x: float, world: int) -> float:
    if not grouped():
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(coda, it, steps: int, world: int) -> float:
    """Exactly `steps` CoDA steps between barrier + synchronize on both sides; max over ranks (s)."""
    torch.cuda.synchronize()
    if grouped():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        x, y = next(it)
        coda.train_step(x, y)
    torch.cuda.synchronize()
    if grouped():
        dist.barrier()
    torch.cuda.synchronize()
    return max_over_ranks(time.perf_counter() - t0, world)


# ----------------------------------------------------------------------------- training legs
def make_coda(arch, batch, image_size, I, pos_ratio, pool, world, rank, device, fused_bn=True, gemm_conv1x1=True,
              graph=False, lr=0.1, flip=0.0, weight_shadow=None):
    from distributedauc_amd.backbone import build_backbone
    from distributedauc_amd.coda import CoDA
    from distributedauc_amd.loader import DeviceLoader, SyntheticImageNet, imagenet_like_labels

    torch.manual_seed(1234)
    split = 499
    labels = imagenet_like_labels(1 << 16, 1000, split, pos_ratio=pos_ratio, seed=123 + rank)
    ds = SyntheticImageNet(labels, image_size, split)
    # bf16 images: the values autocast would cast them to before the stem, cast once per pooled batch
    loader = DeviceLoader(ds, np.arange(len(labels)), batch, device, seed=1234 + rank, channels_last=True, pool=pool,
                          flip=flip, dtype=torch.bfloat16)
    net = build_backbone(arch, num_classes=2).to(device).to(memory_format=torch.channels_last)
    net.set_fused_bn(bool(fused_bn)).set_gemm_conv1x1(bool(gemm_conv1x1))
    coda = CoDA(net, lr=lr, gamma=2000.0, T0=10 ** 9, I=I, split_index=split, world=world, rank=rank,
                autocast_dtype=torch.bfloat16, device=device, collective=grouped(),
                weight_shadow=None if weight_shadow is None else bool(weight_shadow))
    if weight_shadow in (1, 2):
        net.set_weight_shadow(True, dgrad_fwd=weight_shadow == 2, wgrad_hip=False)
    it = iter(loader)
    coda.average_all()            # main.py:141-142
    coda.begin_stage(1, it)       # alpha estimate + anchors (untimed)
    coda.use_graph(graph)         # step bodies replayed from one HIP graph (captured at the first step)
    return coda, it


def bench_train(args, world, rank, device):
    from distributedauc_amd import _lib

    coda, it = make_coda(args.arch, args.batch, args.image_size, args.I, args.pos_ratio, args.pool, world, rank,
                         device, args.fused_bn, args.gemm_conv1x1, lr=args.lr, flip=args.signal_flip,
                         weight_shadow=int(args.weight_shadow))
    if args.graph:
        coda.use_graph(True, eager_update=True)
    log(f"rank {rank}: model + data ready, first steps compile/tune MIOpen kernels")
    lib = _lib.load()
    upd = KernelTimer(lib, "dauc_pd_update")
    sur = KernelTimer(lib, "dauc_surrogate_fwdbwd")
    # the step's BN kernels (csrc/bn_act.hip) timed by HIP events around every call during the last
    # warm-up steps (an event pair per call is host work the timed steps must not pay; the first
    # warm-up step compiles and tunes, so it is never in the window)
    nbn = min(args.bn_steps, max(args.warmup - 1, 0)) if (args.fused_bn and not args.graph) else 0
    bnf = KernelTimer(lib, "dauc_bn_act_forward", bn_forward_bytes)
    bnb = KernelTimer(lib, "dauc_bn_act_backward", bn_backward_bytes)
    for i in range(args.warmup):
        if i == args.warmup - nbn:
            torch.cuda.synchronize()
            bnf.enabled = bnb.enabled = True
        x, y = next(it)
        coda.train_step(x, y)
    bnf.enabled = bnb.enabled = False
    bnf.restore()
    bnb.restore()
    torch.cuda.synchronize()
    bn = None
    if nbn > 0:
        bn = {"steps": nbn, "fwd_ms": bnf.total_ms() / nbn, "bwd_ms": bnb.total_ms() / nbn,
              "calls_per_step": (len(bnf.pairs) + len(bnb.pairs)) / nbn,
              "bytes_per_step": (bnf.bytes + bnb.bytes) / nbn}
    log(f"rank {rank}: warm-up done")
    upd.enabled = sur.enabled = True
    dt = timed_steps(coda, it, args.steps, world)
    upd.enabled = sur.enabled = False
    upd.restore()
    sur.restore()
    loss = float(coda.last_loss.item())
    out = {
        "dt": dt, "imgs": world * args.batch * args.steps, "loss": loss, "n_params": coda.state.numel(),
        "update_ms": upd.mean_ms(), "update_bytes": coda.state.bytes_per_update(True),
        "surrogate_us": (sur.mean_ms() * 1e3) if sur.pairs else None,  # inside the graph: not timed
        "payload_bytes": coda.state.n_reduce * 4, "graph": bool(coda._graph_on),
        "graph_captures": coda.graph_captures, "bn": bn,
    }
    if args.sweep_I:
        out["period_sweep"] = bench_period_sweep(coda, it, args, world)
    if grouped():
        out["coda_round"] = bench_coda_round(coda, world)
    if args.eval_images > 0:
        out["training_eval"] = bench_training_eval(coda, args, world, rank, device)
    del coda, it
    torch.cuda.empty_cache()
    return out


def bench_period_sweep(coda, it, args, world):
    """configs[2]: the same step at each averaging period I (main.py:292-301). Every window is
    --sweep-steps consecutive steps, a multiple of every I, so it holds exactly steps/I rounds."""
    recs = []
    I0 = coda.I
    for I in (int(v) for v in args.sweep_I.split(",") if v.strip()):
        if args.sweep_steps % I:
            raise ValueError(f"--sweep-steps {args.sweep_steps} is not a multiple of I={I}")
        coda.I = I
        dt = timed_steps(coda, it, args.sweep_steps, world)
        recs.append({"I": I, "imgs_per_sec": world * args.batch * args.sweep_steps / dt,
                     "ms_per_step": dt / args.sweep_steps * 1e3, "steps": args.sweep_steps,
                     "rounds_per_step": 1.0 / I, "rounds_in_window": args.sweep_steps // I})
        log(f"rank {coda.rank}: period sweep I={I}: {recs[-1]['ms_per_step']:.2f} ms/step")
    coda.I = I0
    return recs


def bench_training_eval(coda, args, world, rank, device, reps=3):
    """The in-training evaluation (main.py:215-270): the test set scored with rank 0's model, then
    the exact AUC. Split: every rank scores 1/world of the batches after a broadcast of rank 0's
    parameters and BN statistics, all-gather of the scores, sharded count (main.Evaluator). At
    world > 1 the reference's rank-0 scoring is timed beside it.

    MIOpen's default (fast) solvers are not bit-repeatable from call to call, so two scorings of
    the same test set -- split or rank 0, or two repetitions of either -- may differ in the low
    bits of a few scores and flip a near-tie. Bit-identical scoring needs --deterministic_eval
    (61 s for ResNet-50 224^2 bf16 at 8192 images, profiles/r03/final): too slow for the bench.
    So the AUCs of every repetition and of both scoring modes are REPORTED (with their largest
    difference), never asserted equal; tests/test_main_gpu.py checks bit-identity under
    deterministic solvers."""
    from distributedauc_amd.loader import DeviceLoader, SyntheticImageNet, imagenet_like_labels, signal_auc_ceiling
    from distributedauc_amd.main import Evaluator

    n = args.eval_images
    tb = args.batch
    labels = imagenet_like_labels(n, 1000, 499, pos_ratio=args.pos_ratio, seed=777)  # same on every rank
    ds = SyntheticImageNet(labels, args.image_size, 499)
    it = iter(DeviceLoader(ds, np.arange(n), tb, device, seed=777, shuffle=False, channels_last=True,
                           flip=args.signal_flip))
    batches = [next(it) for _ in range((n + tb - 1) // tb)]

    def timed(split):
        ev = Evaluator(batches, n, 499, device, None, world, rank, None, split=split, collective=grouped())
        ev(coda)  # warm (workspaces, MIOpen eval-mode kernels)
        ts, aucs = [], []
        for _ in range(reps):
            if grouped():
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            aucs.append(ev(coda))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return max_over_ranks(float(np.median(ts)), world), aucs

    ms_split, aucs = timed(True)
    rec = {"workload": f"{n} test images {args.image_size}^2 scored by {args.arch} (eval mode, bf16 autocast), "
                       f"test batch {tb}, then the exact AUC; {world} rank(s)",
           "ms": ms_split * 1e3, "imgs_per_sec": n / ms_split, "auc": aucs[-1], "auc_reps": aucs,
           "method": "split" if grouped() else "one rank",
           "auc_note": "AUCs are reported, not asserted equal: MIOpen's fast solvers change low bits between "
                       "scorings (bit-identity needs --deterministic_eval, tested in tests/test_main_gpu.py)"}
    rec["band"] = auc_band(args, n, labels, aucs[-1])
    if grouped():
        ms0, aucs0 = timed(False)
        rec.update({"ms_rank0_scoring": ms0 * 1e3, "speedup_vs_rank0_scoring": ms0 / ms_split,
                    "auc_rank0_scoring": aucs0[-1],
                    "auc_max_abs_diff_split_vs_rank0": max(abs(a - b) for a in aucs for b in aucs0)})
    log(f"rank {rank}: in-training eval of {n} images {ms_split * 1e3:.1f} ms, auc {aucs[-1]:.4f}")
    return rec


def auc_band(args, n, labels, auc):
    """Where the in-training AUC should land: above chance, at most the test set's
    exact Bayes ceiling (the AUC of the sign each image carries, 1 - flip in expectation), next to
    the CPU oracle loop's test AUC on the same workload (scripts/oracle_auc_band.py, committed under
    profiles/r05/; it applies when its configuration is this run's)."""
    from distributedauc_amd.loader import signal_auc_ceiling

    steps_trained = args.warmup + args.steps + (len([v for v in args.sweep_I.split(",") if v.strip()]) * args.sweep_steps
                                                if args.sweep_I else 0)
    ceiling = signal_auc_ceiling(np.arange(n), labels, 499, args.signal_flip)
    rec = {"chance": 0.5, "bayes_ceiling_test_set": ceiling, "flip": args.signal_flip,
           "steps_trained": steps_trained, "cpu_oracle_loop": None}
    f = REPO / "profiles" / "r05" / "oracle_auc_band.json"
    if f.exists():
        o = json.loads(f.read_text())
        c = o.get("config", {})
        same = (c.get("arch"), c.get("batch"), c.get("image_size"), c.get("pool"), c.get("steps"), c.get("lr"),
                c.get("flip"), c.get("test_images")) == (args.arch, args.batch, args.image_size, args.pool,
                                                         steps_trained, args.lr, args.signal_flip, n)
        rec["cpu_oracle_loop"] = {"band": o.get("band"), "same_config": same,
                                  "source": "profiles/r05/oracle_auc_band.json (scripts/oracle_auc_band.py, "
                                            "fp32 torch CPU; not this run)"}
    lo = 0.5 + 0.05  # clearly above chance
    rec["in_band"] = bool(lo <= auc <= ceiling + 0.02)  # + the test set's sampling slack
    rec["band_rule"] = "0.55 <= auc <= bayes_ceiling_test_set + 0.02"
    rec["ceiling_note"] = ("the expected AUC of the best score on this test set (the sign each image carries, "
                           "ties within a sign counted half); a trained model's AUC scatters around it by the "
                           "order it happens to give inside each sign group (sd ~0.006 at 8192 images), hence "
                           "the +0.02 slack")
    return rec


def bench_coda_round(coda, world, reps=5):
    """One CoDA round (main.py:33-54) after the timed steps: the all-reduce of flat[:n_reduce]
    (parameters, a, b, alpha, class counts) + the finalise launch, HIP events on the current stream
    around `reps` rounds (the collective's stream is joined to it), max over ranks. Bus bytes per
    round = 2 (G-1)/G x payload."""
    nbytes = coda.state.n_reduce * 4
    torch.cuda.synchronize()
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.no_grad():
        coda.average_all()  # warm
        e0.record()
        for _ in range(reps):
            coda.average_all()
        e1.record()
    e1.synchronize()
    ms = max_over_ranks(e0.elapsed_time(e1) / reps, world)
    bus = 2 * (world - 1) / world * nbytes / (ms / 1e3) / 1e9
    rec = {"workload": f"all-reduce of {nbytes} B (params + a, b, alpha + class counts) + finalise, {world} ranks",
           "ms_per_round": ms, "payload_bytes": nbytes, "rounds_per_step": 1.0 / coda.I,
           "backend": dist.get_backend(),
           "roofline": {"bound": "xgmi", "achieved": bus, "peak": XGMI_PEAK_GBS, "unit": "GB/s (bus)",
                        "frac": bus / XGMI_PEAK_GBS}}
    if world == 1:
        # the one-rank rehearsal: no bus traffic (the collective is a local copy), so no xGMI figure
        rec["roofline"] = None
        rec["note"] = ("one-rank process group (RCCL rehearsal): the all-reduce moves no bytes over xGMI; "
                       "this times the collective's launch + local copy and the finalise launch")
    return rec


def bench_r18(args, world, rank, device):
    """configs[0] on the GPUs: ResNet-18 CoDA, batch 32 per rank, 224^2, I = 8 (the CPU path of
    the same config is cpu_baseline_configs0)."""
    coda, it = make_coda("resnet18", 32, args.image_size, 8, args.pos_ratio, args.pool, world, rank, device,
                         args.fused_bn, args.gemm_conv1x1, graph=bool(args.r18_graph) and world == 1)
    for _ in range(max(args.warmup, 8)):
        x, y = next(it)
        coda.train_step(x, y)
    torch.cuda.synchronize()
    steps = max(8, args.r18_steps // 8 * 8)
    dt = timed_steps(coda, it, steps, world)
    rec = {"workload": "resnet18 CoDA, batch 32 per rank, 224x224, I=8, bf16 autocast backbone, fp32 AUC kernels "
                       "(BASELINE configs[0] on the GPUs)"
                       + (", step bodies replayed from one HIP graph (averaging rounds eager)" if coda._graph_on else ""),
           "graph": coda._graph_on, "graph_captures": coda.graph_captures,
           "imgs_per_sec": world * 32 * steps / dt, "ms_per_step": dt / steps * 1e3, "steps": steps,
           "n_gpus": world, "params": coda.state.numel(), "final_loss": float(coda.last_loss.item())}
    del coda, it
    torch.cuda.empty_cache()
    return rec


# ----------------------------------------------------------------------------- exact AUC legs
def bench_auc(args, world, rank, device, log2n=None, pos=None, pair_reps=None):
    """configs[3] (and [4]): exact AUC of 2^k scores, sharded over the ranks; both exact methods."""
    from distributedauc_amd import _lib
    from distributedauc_amd.auc import ExactAUC
    from distributedauc_amd.loader import synthetic_scores

    log2n = args.auc_log2n if log2n is None else log2n
    pos = args.auc_pos if pos is None else pos
    n = 1 << log2n
    s, y = synthetic_scores(n, pos, device)  # same scores on every rank
    out = {"n": n, "log2n": log2n, "pos": pos}
    # the sort method: the whole evaluation on one GPU (or below SHARD_MIN) is ONE blocking C call,
    # dauc_auc_eval_counts; over ranks each compacts its slice of the labels
    # (dauc_auc_eval_compact_part), one all-gather of the slots, each counts its query range
    # (dauc_auc_eval_query_part, timed here), one all-gather of the records and one host read
    shard_min = ExactAUC.SHARD_MIN if args.auc_shard_min is None else args.auc_shard_min
    sort_fn = "dauc_auc_eval_counts" if not grouped() or n < shard_min else "dauc_auc_eval_query_part"
    for method, fn in (("sort", sort_fn), ("pairs", "dauc_pair_count")):
        ev = ExactAUC(world=world, rank=rank, variant=args.variant, method=method, shard_min=shard_min,
                      collective=grouped())
        kt = KernelTimer(_lib.load(), fn)
        cold = None
        if method == "sort":
            # the first call ever on this device and stream: the evaluator's workspace and the
            # page-locked readback words are allocated inside it
            torch.cuda.synchronize()
            if grouped():
                dist.barrier()
            t0 = time.perf_counter()
            ev.counts(y, s)
            torch.cuda.synchronize()
            cold = max_over_ranks(time.perf_counter() - t0, world)
        c = ev.counts(y, s)  # warm-up
        reps = (args.auc_reps if pair_reps is None else pair_reps) if method == "pairs" else 5 * args.auc_reps
        # wall time without the event wrapper (its event creation and records are host work of
        # their own), then the same calls again with HIP events around the C entry point
        times = []
        for _ in range(reps):
            torch.cuda.synchronize()
            if grouped():
                dist.barrier()
            t0 = time.perf_counter()
            c = ev.counts(y, s)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        kt.enabled = True
        for _ in range(reps):
            if grouped():
                dist.barrier()
            ev.counts(y, s)
        kt.enabled = False
        kt.restore()
        out["m_" + method] = {"t_eval": max_over_ranks(float(np.median(times)), world),
                              "t_count": max_over_ranks(kt.mean_ms() / 1e3, world), "count_fn": fn, "counts": c,
                              "mode": ev.last_mode}
        if method == "sort":
            # another test set of the same length (other P) alternating with this one: the
            # evaluation keeps no state between calls, so every call does the same work
            g2 = torch.Generator(device=device).manual_seed(4242)
            s2 = torch.rand(n, device=device, generator=g2)
            y2 = torch.where(torch.rand(n, device=device, generator=g2) < pos * 1.1, 1, -1).to(torch.int8)
            alt = []
            for k in range(reps):
                torch.cuda.synchronize()
                if grouped():
                    dist.barrier()
                t0 = time.perf_counter()
                ev.counts(y2, s2) if k % 2 == 0 else ev.counts(y, s)
                torch.cuda.synchronize()
                alt.append(time.perf_counter() - t0)
            out["m_sort"]["t_cold"] = cold
            out["m_sort"]["t_alternating"] = max_over_ranks(float(np.median(alt)), world)
            del s2, y2
            # the same scores rounded to bf16 (a bf16 model's scores: few distinct values, many
            # positives on each): the count index refuses the table and the evaluation runs the
            # sorted path's distinct-key index; checked against one pair-count evaluation of them
            sb = s.bfloat16().float()
            cb = ev.counts(y, sb)
            tb = []
            for _ in range(reps):
                torch.cuda.synchronize()
                if grouped():
                    dist.barrier()
                t0 = time.perf_counter()
                ev.counts(y, sb)
                torch.cuda.synchronize()
                tb.append(time.perf_counter() - t0)
            pb = ExactAUC(world=world, rank=rank, variant=args.variant, method="pairs", shard_min=shard_min,
                          collective=grouped()).counts(y, sb)
            out["m_sort"]["tie_heavy"] = {
                "t_eval": max_over_ranks(float(np.median(tb)), world),
                "distinct_positive_values": int(torch.unique(sb[y == 1]).numel()),
                "counts_match_pair_count": (cb["wins"], cb["ties"]) == (pb["wins"], pb["ties"])}
            if not out["m_sort"]["tie_heavy"]["counts_match_pair_count"]:
                raise RuntimeError(f"exact AUC methods disagree on bf16-rounded scores: {cb} vs {pb}")
            del sb
        log(f"rank {rank}: auc 2^{log2n} {method} eval {out['m_' + method]['t_eval'] * 1e3:.2f} ms")
    a, b = out["m_sort"]["counts"], out["m_pairs"]["counts"]
    if (a["wins"], a["ties"]) != (b["wins"], b["ties"]):
        raise RuntimeError(f"exact AUC methods disagree: {a} vs {b}")
    out.update({"P": a["P"], "N": a["N"], "wins": a["wins"], "ties": a["ties"], "auc": ExactAUC.from_counts(a),
                "npairs": a["P"] * a["N"]})
    if rank == 0 and cpu_baseline_on(args, world):
        out["scores_host"] = (s.cpu().numpy(), y.cpu().numpy().astype(np.int64))
    return out


def cpu_baseline_on(args, world: int) -> bool:
    """The CPU baselines run at N = 1 (the bench contract), or at any N with --cpu-baseline-any-n."""
    return not args.no_cpu_baseline and (world == 1 or args.cpu_baseline_any_n)


def auc_record(auc, world, config_name):
    pk, sk = auc["m_pairs"], auc["m_sort"]
    npairs = auc["npairs"]
    pc_rate = npairs / pk["t_count"]
    n = auc["n"]
    # the sort method's HBM floor: labels read once by the compaction, scores + labels once by the
    # query pass, each over the rank's share when sharded (the positives' scores, the gathered
    # slots and the count index are ~0.1-1 % of that)
    shard = world if sk["mode"] == "sharded" else 1
    eval_bytes = n * 1 // shard + n * (4 + 1) // shard
    return {
        "workload": f"exact AUC, 2^{auc['log2n']} fp32 scores, {auc['pos']:.1%} positives "
                    f"(BASELINE {config_name}), {world} rank(s); sort method {sk['mode']} "
                    "(sharded = every rank compacts the positives of its slice of the labels, one all-gather of "
                    "the slots, every rank builds the index from the gathered positives and counts its score-index "
                    "range, one all-gather of the 8-word part records; replicated = every rank evaluates the whole "
                    "vector, below 2^24 scores); pair count: positive blocks, int64 all-reduce",
        "sort_mode": sk["mode"],
        # north_star's pair-compare throughput: the pair-count kernel, which compares every
        # positive with every negative (its roofline below)
        "pair_compare_per_sec": pc_rate,
        # the sort method enumerates no pairs: P*N / its wall time is an EFFECTIVE rate only
        "effective_pairs_per_sec": npairs / sk["t_eval"],
        "effective_pairs_what": "P*N / the sort method's evaluation wall time: it locates each negative among the "
                                "positives and compares no pairs, so this exceeds any pair-compare ceiling",
        "method": "sort (default evaluator: compact the positives reading labels only, build the LDS count index "
                  "straight from them with the table size read on the device (cell-ordered table, no sort), locate "
                  "every negative, read in place, through it -- all enqueued with no host sync; one readback per "
                  "call; for tables the index does not fit or finds skewed, the radix sort and behind it the LDS "
                  "distinct-key index (tie-heavy tables, up to 14,000 distinct keys) or the LDS search tree)",
        "eval_ms": sk["t_eval"] * 1e3, "sort_count_ms": sk["t_count"] * 1e3,
        "eval_ms_cold": sk["t_cold"] * 1e3,
        "eval_ms_cold_what": "the first call on this device/stream: workspace + page-locked readback words allocated",
        "eval_ms_other_data": sk["t_alternating"] * 1e3,
        "eval_ms_tie_heavy": sk["tie_heavy"]["t_eval"] * 1e3,
        "eval_tie_heavy_what": (f"the same scores rounded to bf16 ({sk['tie_heavy']['distinct_positive_values']} "
                                "distinct positive values; a bf16 model's scores): the count index refuses the "
                                "table, the blocking call runs the sorted path's LDS distinct-key index; counts "
                                "equal the pair count's on the same scores: "
                                f"{sk['tie_heavy']['counts_match_pair_count']}"),
        "eval_ms_other_data_what": "median over calls alternating with another test set of the same length and a "
                                   "different P (no state between calls: no speculation, no miss path)",
        "sort_count_what": f"HIP events around every {sk['count_fn']} call"
                           + (" (the whole one-call evaluation: compaction, index build, query, readback)"
                              if sk["count_fn"] == "dauc_auc_eval_counts" else
                              " (this rank's step 2: the gathered slots' table, index build, its query share, record "
                              "copy; its slice's compaction and the two all-gathers are in eval_ms)"),
        "eval_roofline": {"bound": "hbm", "bytes_per_rank": eval_bytes,
                          "achieved": eval_bytes / sk["t_eval"] / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": eval_bytes / sk["t_eval"] / 1e9 / HBM_PEAK_GBS,
                          "note": "bytes = 1 label pass + 1 score/label pass over this rank's share (all n at N=1)"},
        "query_kernel": load_profile("query_valu.json", f"2^{auc['log2n']}"),
        "P": auc["P"], "N": auc["N"], "wins": auc["wins"], "ties": auc["ties"], "auc": auc["auc"],
        "methods_agree": True,
        "pair_count_kernel": {
            "pairs_per_sec": pc_rate, "eval_ms": pk["t_eval"] * 1e3, "count_ms": pk["t_count"] * 1e3,
            "roofline": {"kernel": "dauc_pair_count", "bound": "valu", "achieved": pc_rate / world,
                         "peak": VALU_PAIR_PEAK, "unit": "pairs/s per GPU",
                         "frac": pc_rate / world / VALU_PAIR_PEAK,
                         "peak_note": "packed-issue ceiling: 3 fp32 lane-ops per pair on 32-wide SIMDs",
                         "survey_peak": SURVEY_PAIR_PEAK, "frac_vs_survey_peak": pc_rate / world / SURVEY_PAIR_PEAK,
                         "survey_peak_note": "SURVEY §8(d): 2 compares per pair on 16-wide SIMDs"}},
    }


# ----------------------------------------------------------------------------- loss kernel leg
def bench_surrogate(args, device):
    """The fused loss kernel at a streaming size (9 B/element = fp32 h + int8 y + fp32 dh).

    Training batches (B = 256) are launch-latency bound; this leg measures the same kernel where
    HBM bounds it. Inputs resident in HBM. Reported separately: the whole ABI call (ONE launch:
    the stream and its row reduce), and from the tuning build the streaming kernel alone and the
    same launch's stream without its reduce (include/dauc_tuning.h variants 3 and 4)."""
    from distributedauc_amd import _lib, ops

    B = 1 << args.sur_log2b
    g = torch.Generator(device=device).manual_seed(7)
    h = torch.rand(B, device=device, generator=g)
    y = torch.where(torch.rand(B, device=device, generator=g) < args.pos_ratio, 1, -1).to(torch.int8)
    abalpha = torch.tensor([0.1, -0.2, 0.3], device=device)
    p_hat = torch.tensor([args.pos_ratio], device=device)
    dh = torch.empty(B, device=device)
    grad3 = torch.empty(3, device=device)
    out64 = torch.zeros(6, dtype=torch.float64, device=device)

    def b2b(variant):
        # warm: the first ~200-300 calls of a streaming kernel run 2-4 us slower than the steady
        # state (profiles/r02/surrogate_tail/sur_order_effect.jsonl); 400 calls is ~40 ms
        for _ in range(max(400, 4 * args.sur_reps)):
            ops.surrogate_fwdbwd(h, y, abalpha, p_hat, dh=dh, grad3=grad3, out64=out64, variant=variant)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.sur_reps):
            ops.surrogate_fwdbwd(h, y, abalpha, p_hat, dh=dh, grad3=grad3, out64=out64, variant=variant)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / args.sur_reps

    # (1) HIP events over the timed region: one pair around sur_reps back-to-back calls on the
    #     launch stream (the average includes the gaps between calls, not per-call event packets)
    ms = b2b(0)
    loss = float(out64[0].item())
    # the tuning build's stream alone (variant 3: no hand-off, no reduce) and the product
    # kernel's stream with its tagged row stores but nobody reducing (variant 22)
    stream_ms = b2b(3)
    tail_stream_ms = b2b(22)
    # (2) an event pair around every call (each pair adds its own marker packets to the stream)
    kt = KernelTimer(_lib.load(), "dauc_surrogate_fwdbwd")
    kt.enabled = True
    for _ in range(args.sur_reps):
        ops.surrogate_fwdbwd(h, y, abalpha, p_hat, dh=dh, grad3=grad3, out64=out64)
    kt.enabled = False
    kt.restore()
    per_call_ms = kt.mean_ms()
    # every reduction of the leg completed (a timed-out one would have returned NaN: VERDICT r04 #4)
    status = ops.surrogate_status(device, raise_on_error=True)
    nbytes = 9 * B
    gbs = nbytes / (ms / 1e3) / 1e9
    sgbs = nbytes / (stream_ms / 1e3) / 1e9
    return {"workload": f"fused surrogate fwd+bwd, B = 2^{args.sur_log2b} fp32 scores, int8 labels, p = {args.pos_ratio}",
            "B": B, "avg_launch_us": ms * 1e3, "per_call_events_us": per_call_ms * 1e3,
            "timing": f"HIP events around {args.sur_reps} back-to-back calls on the launch stream, divided by the "
                      "call count (per_call_events_us: an event pair around every call instead)",
            "loss": loss, "reduction_status": status,
            "roofline": {"kernel": "dauc_surrogate_fwdbwd (whole call)", "launches": "surrogate_tail_x_kernel: the stream "
                         "and its fp64 row reduce (by 128 extra workgroups that stream nothing, the last one taking "
                         "the grid's last 512 rows itself; epoch-tagged granules) in ONE launch",
                         "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "traffic": load_traffic(f"surrogate_2^{args.sur_log2b}"),
                         "bytes_per_launch": nbytes},
            "stream_kernel": {"kernel": "surrogate_chunk_kernel alone (tuning variant 3: no row reduce, no scalars)",
                              "avg_launch_us": stream_ms * 1e3, "bound": "hbm", "achieved": sgbs,
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": sgbs / HBM_PEAK_GBS,
                              "bytes_per_launch": nbytes},
            "tail_stream_us": tail_stream_ms * 1e3,
            "tail_stream_what": "the product kernel's stream with its tagged row stores, its reducers returning at "
                                "once (variant 22)",
            "row_reduce_us": (ms - tail_stream_ms) * 1e3,
            "row_reduce_what": "whole call - variant 22: the in-launch hand-off chain after the last row lands"}


def step_roofline(args, res) -> dict:
    """The roofline of what `value` measures: the whole training step against the bf16 dense MFMA
    peak (convolution + fc FLOP from the layer shapes), and its BN passes against HBM (bytes per call
    from bn_forward_bytes / bn_backward_bytes, time by HIP events around every BN call in
    res["bn"]'s window of warm-up steps) -- VERDICT r05 #2."""
    ms = res["dt"] / args.steps * 1e3
    fl = backbone_flops(args.arch, args.image_size, args.batch)
    tf = fl["flop_per_step"] / (ms / 1e3) / 1e12
    rec = {"bound": "mfma", "flop_per_step": fl["flop_per_step"], "forward_gmac": fl["forward_gmac"],
           "achieved": tf, "peak": MFMA_BF16_PEAK_TFS, "unit": "TFLOP/s", "frac": tf / MFMA_BF16_PEAK_TFS,
           "per_rank": True,
           "what": f"{args.arch} b{args.batch} {args.image_size}^2 per rank: conv + fc FLOP (forward 2 MAC, weight "
                   "gradient 2 MAC, input gradient 2 MAC except the stem's) / ms_per_step, against the bf16 dense "
                   "MFMA peak (MI355X_MICROARCH.md); the step also runs BN, pooling and the AUC kernels, which are "
                   "HBM work (bn below; roofline = the update kernel)"}
    bn = res.get("bn")
    if bn:
        bms = bn["fwd_ms"] + bn["bwd_ms"]
        gbs = bn["bytes_per_step"] / (bms / 1e3) / 1e9 if bms > 0 else float("nan")
        rec["bn"] = {"bound": "hbm", "bytes_per_step": bn["bytes_per_step"], "ms_per_step": bms,
                     "fwd_ms": bn["fwd_ms"], "bwd_ms": bn["bwd_ms"], "calls_per_step": bn["calls_per_step"],
                     "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                     "share_of_step": bms / ms, "steps_timed": bn["steps"],
                     "what": "fused BN + add + ReLU (csrc/bn_act.hip): algorithmic bytes of its two passes each way "
                             "(forward: stats read x, apply read x [+ residual] write y [+ 1-bit mask]; backward: reduce "
                             "read dy + mask + x [write dz], dx read dy + mask | dz + x write dx) / the summed HIP-event "
                             "time of every BN call (all its launches, finalizes included), in a window of "
                             f"the last {bn['steps']} warm-up steps (untimed)"}
    return rec


# ----------------------------------------------------------------------------- CPU baselines
def cpu_baseline_train_cores(args, host):
    """configs[1]'s CPU path at the thread budget (OMP_NUM_THREADS, the box's CPU share) and at every
    CPU of the affinity mask; `value` is the faster. The all-CPU leg runs in a child
    process that never touches the GPU, killed after 2 x --cpu-max-s (a bounded sample: on a host
    whose cgroup quota is below the affinity mask, that many threads oversubscribe the quota)."""
    runs = [cpu_baseline_train(args, host["cpu_budget"])]
    more = all_cores_leg(host)
    if isinstance(more, int):
        log(f"cpu baseline: {args.arch} step at {more} threads (every usable CPU; child process)")
        runs.append(cpu_train_child(args, more, timeout=2 * args.cpu_max_s))
    else:
        runs.append({"cores": host["affinity_cpus"], "skipped": more})
    torch.set_num_threads(host["cpu_budget"])
    done = [r for r in runs if "value" in r]
    best = dict(max(done, key=lambda r: r["value"]))
    best["by_threads"] = runs
    best["cores_note"] = (f"timed at {host['cpu_budget']} threads (the budget); nproc {host['nproc']}, affinity mask "
                          f"{host['affinity_cpus']} CPUs, cgroup quota {host.get('cgroup_cpu_quota')} CPUs; value = the "
                          "fastest leg")
    return best


def all_cores_leg(host):
    """Threads for the every-CPU leg of the CPU baselines, or why it is not run: the
    CPUs of time the process can get are the affinity mask capped by the cgroup quota. On the GPU box
    the quota is 16 CPUs under a 256-CPU mask, and threads past it oversubscribe the quota: ResNet-50
    b32 took 2.0x as long at 64 threads as at 16, and at 256 threads did not finish one step in 180 s
    (profiles/r06/host_cores/)."""
    usable = host.get("usable_cpus", host["affinity_cpus"])
    if usable > host["cpu_budget"]:
        return usable
    return (f"not run: the cgroup quota ({host.get('cgroup_cpu_quota')} CPUs) caps this process below its "
            f"{host['affinity_cpus']}-CPU affinity mask, so the budget of {host['cpu_budget']} threads is every CPU it "
            "can use; more threads oversubscribe the quota (64 threads: 2.0x slower than 16, 256 threads: no "
            "ResNet-50 step in 180 s, profiles/r06/host_cores/)")


def cpu_train_child(args, threads, timeout):
    """cpu_baseline_train(args, threads) in a child process (HIP hidden: it never touches the GPU),
    killed after `timeout` seconds; its record, or why there is none."""
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "cpu_train.json"
        env = {k: v for k, v in os.environ.items() if not (k.startswith("TORCHELASTIC_") or k in _LAUNCH_VARS)}
        env.update(HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="", OMP_NUM_THREADS=str(threads))
        cmd = [sys.executable, str(Path(__file__).resolve()), "--cpu-train-worker", "--cw-threads", str(threads),
               "--cw-out", str(out), "--arch", args.arch, "--batch", str(args.batch), "--image-size",
               str(args.image_size), "--pos-ratio", str(args.pos_ratio), "--cpu-max-s", str(args.cpu_max_s)]
        proc = subprocess.Popen(cmd, env=env)
        try:
            rc = proc.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
            return {"cores": threads, "skipped": f"not done within {timeout:.0f} s (a bounded sample)"}
        if rc != 0 or not out.exists():
            return {"cores": threads, "skipped": f"child exited with {rc}"}
        return json.loads(out.read_text())


def cpu_baseline_train(args, threads, max_s=None):
    """The reference's CPU path for the headline config: torch-CPU ResNet-50 fwd at the GPU's batch
    (256, 224^2), verbatim loss (main.py:313-317), autograd, per-tensor dppd_sg (main.py:56-64)
    + running average (main.py:333-334). One warm-up step at batch 32, one timed step at 256."""
    from distributedauc_amd.backbone import build_backbone
    from oracle import reference_cpu as R

    torch.set_num_threads(threads)
    torch.manual_seed(0)
    B = args.batch
    net = build_backbone(args.arch, num_classes=2)
    net0 = {k: v.clone() for k, v in net.state_dict().items()}
    avg = {k: v.clone() for k, v in net.state_dict().items()}
    a, b, alpha = (torch.zeros(1, requires_grad=True) for _ in range(3))
    p = torch.tensor([args.pos_ratio])

    def step(nb):
        x = torch.randn(nb, 3, args.image_size, args.image_size)
        lab = torch.where(torch.rand(nb) < args.pos_ratio, 1, -1)
        h = net(x)[:, 1]
        loss = R.surrogate_loss(h, lab, a, b, alpha, p)
        net.zero_grad()
        loss.backward()
        with torch.no_grad():
            for name, prm in net.named_parameters():
                prm.data = R.pd_step(prm.data, prm.grad.data, net0[name], 0.1, 2000.0)
                avg[name] = avg[name] + prm.data

    t0 = time.perf_counter()
    step(32)  # warm-up
    t32 = time.perf_counter() - t0
    if max_s is not None and t32 * B / 32 > max_s:
        return {"cores": threads, "skipped": f"warm-up at batch 32 took {t32:.1f} s: the batch-{B} step would take "
                                             f"~{t32 * B / 32:.0f} s > {max_s} s", "warmup_s": t32}
    t0 = time.perf_counter()
    step(B)
    dt = time.perf_counter() - t0
    return {"value": B / dt, "unit": "imgs/sec", "cores": threads, "kind": "port", "warmup_s": t32,
            "sample": f"{args.arch} {args.image_size}x{args.image_size}, one timed step at batch {B} (the GPU's "
                      "batch; warm-up at 32): fwd + reference loss + backward + per-tensor dppd_sg + running "
                      f"average, torch CPU fp32, {threads} threads", "seconds": dt}


def cpu_coda_worker(args):
    """One rank of the configs[0] CPU baseline (ResNet-18 b32 224^2, I=8): the reference's step
    restated by the oracle (main.py:303-334) with average_all over gloo (main.py:33-54, 292-301).
    Never touches the GPU. Rank 0 writes the timings as JSON to --cw-out."""
    from distributedauc_amd.backbone import build_backbone
    from oracle import reference_cpu as R

    torch.set_num_threads(max(1, args.cw_threads))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(args.cw_port)
    world = args.cpu_workers
    dist.init_process_group("gloo", rank=args.cw_rank, world_size=world)
    torch.manual_seed(1234)
    net = build_backbone("resnet18", num_classes=2)
    net0 = {k: v.clone() for k, v in net.state_dict().items()}
    avg = {k: v.clone() for k, v in net.state_dict().items()}
    a, b, alpha = (torch.zeros(1, requires_grad=True) for _ in range(3))
    gpos, gneg = torch.zeros(1), torch.zeros(1)
    lpos, lneg = torch.zeros(1), torch.zeros(1)
    gen = torch.Generator().manual_seed(1234 + args.cw_rank)
    B, I = 32, 8

    def step(t_total):
        nonlocal lpos, lneg
        if t_total % I == 0:  # main.py:292-301
            with torch.no_grad():
                R.average_all_dist(net, a, b, alpha, gpos, gneg, lpos, lneg, world)
            lpos, lneg = torch.zeros(1), torch.zeros(1)
        x = torch.randn(B, 3, args.image_size, args.image_size, generator=gen)
        lab = torch.where(torch.rand(B, generator=gen) < args.pos_ratio, 1, -1)
        lpos += float((lab == 1).sum())
        lneg += float((lab == -1).sum())
        p = torch.tensor([float(gpos + lpos) / float(gpos + lpos + gneg + lneg)])  # main.py:309-310
        h = net(x)[:, 1]
        loss = R.surrogate_loss(h, lab, a, b, alpha, p)
        net.zero_grad()
        a.grad = b.grad = alpha.grad = None
        loss.backward()
        with torch.no_grad():
            for name, prm in net.named_parameters():
                prm.data = R.pd_step(prm.data, prm.grad.data, net0[name], 0.1, 2000.0)
                avg[name] = avg[name] + prm.data

    with torch.no_grad():
        R.average_all_dist(net, a, b, alpha, gpos, gneg, lpos, lneg, world)  # main.py:141-142
    t = 1
    step(t)  # warm-up
    t += 1
    while t % I:  # align so the timed window holds exactly steps / I rounds
        t += 1
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        step(t)
        t += 1
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    # the averaging round alone (the survey measured 127.9 ms for R-18 on 4 ranks)
    rounds = 3
    dist.barrier()
    t0 = time.perf_counter()
    with torch.no_grad():
        for _ in range(rounds):
            R.average_all_dist(net, a, b, alpha, gpos, gneg, lpos, lneg, world)
    dist.barrier()
    dr = torch.tensor([(time.perf_counter() - t0) / rounds], dtype=torch.float64)
    dist.all_reduce(dr, op=dist.ReduceOp.MAX)
    if args.cw_rank == 0 and args.cw_out:
        nparams = sum(p.numel() for p in net.parameters())
        Path(args.cw_out).write_text(json.dumps({
            "dt": float(dt), "steps": args.cpu_steps, "imgs": world * B * args.cpu_steps,
            "round_ms": float(dr) * 1e3, "params": nparams,
            "params_finite": all(bool(torch.isfinite(p).all()) for p in net.parameters())}))
    dist.destroy_process_group()


_LAUNCH_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")


def cpu_baseline_configs0(args, host, threads_total=None, timeout=600):
    """configs[0]: 4 gloo CPU worker processes x (budget / 4) threads, ResNet-18 b32 224^2, I = 8
    ("4 processes x nproc/4 threads"). Child processes of this one (they never touch
    the GPU); their rank 0 reports the max-over-ranks time of exactly --cpu-steps steps."""
    W = args.cpu_workers
    threads = max(1, (threads_total or host["cpu_budget"]) // W)
    port = free_port()
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "cw.json"
        # a job of their own: none of this rank's launcher variables (under torch.distributed.run,
        # TORCHELASTIC_USE_AGENT_STORE would make their rendezvous wait for the agent's store)
        env = {k: v for k, v in os.environ.items()
               if not (k.startswith("TORCHELASTIC_") or k in _LAUNCH_VARS)}
        env.update(HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="",
                   OMP_NUM_THREADS=str(threads), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs = [subprocess.Popen([sys.executable, str(Path(__file__).resolve()), "--cpu-coda-worker",
                                   "--cpu-workers", str(W), "--cw-rank", str(r), "--cw-port", str(port),
                                   "--cw-threads", str(threads), "--cw-out", str(out),
                                   "--cpu-steps", str(args.cpu_steps), "--image-size", str(args.image_size),
                                   "--pos-ratio", str(args.pos_ratio)], env=env)
                 for r in range(W)]
        try:
            rcs = [p.wait(timeout=timeout) for p in procs]
        except subprocess.TimeoutExpired:
            return {"cores": W * threads, "workers": W, "threads_per_worker": threads,
                    "skipped": f"not done within {timeout} s (a bounded sample)"}
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        if any(rcs) or not out.exists():
            return {"error": f"cpu workers exited with {rcs}"}
        r = json.loads(out.read_text())
    return {"value": r["imgs"] / r["dt"], "unit": "imgs/sec", "cores": W * threads, "kind": "port",
            "workers": W, "threads_per_worker": threads, "ms_per_step": r["dt"] / r["steps"] * 1e3,
            "averaging_round_ms": r["round_ms"], "params": r["params"], "params_finite": r["params_finite"],
            "sample": f"resnet18 {args.image_size}x{args.image_size} batch 32 per worker, I=8, {W} gloo worker processes x {threads} threads, "
                      f"{r['steps']} timed steps (one averaging round inside: per-parameter all_reduce + /= size, "
                      "main.py:33-54), fwd + reference loss + backward + per-tensor dppd_sg + running average, "
                      "torch CPU fp32"}


def cpu_baseline_auc(auc_res, max_log2n=None, oracle_check=False):
    """sklearn roc_curve + auc (main.py:79-81) on the same scores: the reference CPU path, and
    (oracle_check) the C oracle's integer counts on the full vector vs the GPU's."""
    from oracle import reference_cpu as R

    s, y = auc_res["scores_host"]
    n = s.size
    rec = {}
    if oracle_check:
        from oracle import coracle

        t0 = time.perf_counter()
        e = coracle.auc_counts(y, s)
        rec["oracle_counts"] = {"wins": e["wins"], "ties": e["ties"], "P": e["P"], "N": e["N"],
                                "seconds": time.perf_counter() - t0,
                                "match": (e["wins"], e["ties"], e["P"], e["N"]) ==
                                         (auc_res["wins"], auc_res["ties"], auc_res["P"], auc_res["N"]),
                                "what": "C restatement of sklearn _binary_clf_curve's integer counts "
                                        "(oracle/auc_oracle.c) on the full vector, vs the GPU counts"}
    if max_log2n is not None and n > (1 << max_log2n):
        s, y = s[:1 << max_log2n], y[:1 << max_log2n]
    P = int(np.sum(y == 1))
    t0 = time.perf_counter()
    ref = R.auc_sklearn(y, s)
    dt = time.perf_counter() - t0
    full = s.size == n
    rec.update({"value": P * (s.size - P) / dt, "unit": "pairs/sec (effective: P*N / wall)", "cores": 1,
                "kind": "port", "seconds": dt, "auc": ref,
                "sample": (f"full 2^{int(np.log2(n))} scores" if full else
                           f"first 2^{int(np.log2(s.size))} of the 2^{int(np.log2(n))} scores") +
                          ", sklearn roc_curve+auc (single-threaded sort)"})
    if full:
        rec["auc_abs_diff"] = abs(ref - auc_res["auc"])
    return rec


# ----------------------------------------------------------------------------- launch
def self_launch(args) -> int | None:
    """--gpus N without a launcher: start N ranks as a torch.distributed.run child process (this
    process has not touched the GPU) and return its exit code."""
    if args.cpu_coda_worker or args.cpu_train_worker or "WORLD_SIZE" in os.environ or (
            args.gpus <= 1 and args.backend is None):
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve()), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"launching {args.gpus} rank(s): {' '.join(cmd[1:5])} ...")
    return subprocess.call(cmd, env=env)


def gemm_selections(path: str) -> None:
    """Read-only TunableOp selections for the 1x1 convolutions' GEMMs (scripts/tune_gemms.py: tuned
    with every candidate checked against the default solution; the shipped file
    distributedauc_amd/tunableop_gfx950.csv, profiles/r05/tunableop/); no tuning at run time, so every
    rank and run uses the same solutions. DAUC_TUNABLEOP=0 (or a missing file): the default solutions.
    The file's validators (torch, HIP, hipBLASLt, rocBLAS versions, gfx950) must match, else torch
    ignores its entries."""
    if not path or path == "0" or not os.path.exists(path):
        return
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.set_filename(path)
    tunable.read_file(path)


def main():
    args = parse()
    if args.cpu_coda_worker:
        cpu_coda_worker(args)
        return
    if args.cpu_train_worker:  # one CPU baseline leg in a child process (cpu_train_child)
        Path(args.cw_out).write_text(json.dumps(cpu_baseline_train(args, args.cw_threads, max_s=args.cpu_max_s)))
        return
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    if int(os.environ.get("RANK", "0")) == 0:
        start_heartbeat()
    # Only the JSON record goes to stdout: everything else written to fd 1 (gloo's C++ connection
    # messages, CPU worker children, library chatter) is sent to stderr for the rest of the run.
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    ndev = torch.cuda.device_count()
    backend = args.backend or "nccl"
    use_group = world > 1 or args.backend is not None
    if backend == "nccl" and world > 1 and ndev < local_world:
        print(f"error: the nccl (RCCL) backend needs one GPU per rank: {local_world} ranks on this node, "
              f"{ndev} GPU(s) visible (use --backend gloo for a shared-GPU rehearsal)", file=sys.stderr)
        sys.exit(3)
    device = torch.device("cuda", local % max(ndev, 1))  # ranks share a device only in gloo rehearsals
    torch.cuda.set_device(device)
    shared = local_world > max(ndev, 1)  # gloo rehearsal: several ranks on one GPU
    gemm_sel = "off: ranks share a GPU" if shared else (
        "off: DAUC_TUNABLEOP=0" if os.environ.get("DAUC_TUNABLEOP") == "0" else "shipped TunableOp selections")
    if shared:
        # the selections were tuned and checked with one process owning the GPU; the first 8-rank
        # shared-GPU rehearsal with them on (round 6) aborted in one rank with an illegal-instruction
        # fault in a hipBLASLt GEMM (profiles/r06/n8_gloo_fault/README.txt) -- a shared GPU takes the
        # default solutions; one rank per GPU (the driver's N > 1 run, and N = 1) keeps them
        log(f"rank {rank}: {local_world} ranks share {ndev} GPU(s): TunableOp selections off (default GEMM solutions)")
    else:
        gemm_selections(os.environ.get("DAUC_TUNABLEOP", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                        "distributedauc_amd", "tunableop_gfx950.csv")))
    quiet = None
    if use_group:
        if "MASTER_ADDR" not in os.environ:  # a --backend run at --gpus 1 outside a launcher
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            print(f"error: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}", file=sys.stderr)
            sys.exit(2)
        quiet = dist.new_group(backend="gloo")  # waits without spinning a core (CPU baseline runs on rank 0)
    host = host_info()

    res = bench_train(args, world, rank, device) if not args.no_train else None
    r18 = bench_r18(args, world, rank, device) if (not args.no_train and args.r18_steps > 0) else None
    auc = bench_auc(args, world, rank, device) if not args.no_auc else None
    auc2 = None
    if not args.no_auc and args.auc2_log2n > 0:  # configs[4]: 2^27 scores at 0.1 % positives
        auc2 = bench_auc(args, world, rank, device, args.auc2_log2n, args.auc2_pos, pair_reps=1)
    sur = bench_surrogate(args, device) if (not args.no_surrogate and rank == 0) else None
    torch.cuda.synchronize()

    if rank == 0:
        out = {"metric": METRIC, "n_gpus": world}
        if res is not None:
            upd_gbs = res["update_bytes"] / (res["update_ms"] / 1e3) / 1e9
            out.update({
                "value": res["imgs"] / res["dt"], "unit": "imgs/sec", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": res["dt"] / args.steps * 1e3, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "auc_kernels_dtype": "f32",
                "dtype_what": "bf16 = the backbone's arithmetic (autocast convolutions / GEMMs, fp32 accumulation, "
                              "fp32 master weights); the AUC loss, update and exact-AUC kernels compute in fp32",
                "data": "synthetic",
                "config": {"workload": f"{args.arch} CoDA, bf16 autocast backbone"
                                       f"{' (fused BN+add+ReLU kernels)' if args.fused_bn else ''}"
                                       f"{' (1x1 convs as GEMMs)' if args.gemm_conv1x1 else ''}, fp32 AUC kernels "
                                       "(BASELINE configs[1])",
                           "global_batch": args.batch * world, "image_size": args.image_size, "I": args.I,
                           "lr": args.lr, "gamma": 2000.0, "signal_flip": args.signal_flip,
                           "pos_ratio": args.pos_ratio, "parallelism": f"dp{world}", "params": res["n_params"]},
                "roofline": {"kernel": "dauc_pd_update (fused dppd_sg + running average)", "bound": "hbm",
                             "achieved": upd_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": upd_gbs / HBM_PEAK_GBS, "traffic": load_traffic("pd_update"),
                             "bytes_per_launch": res["update_bytes"], "avg_launch_us": res["update_ms"] * 1e3},
                "step_roofline": step_roofline(args, res),
                "surrogate_us_per_call": res["surrogate_us"],
                "step_graph": {"replayed": res["graph"], "captures": res["graph_captures"],
                               "what": "label map -> forward -> surrogate -> backward replayed from one HIP graph; "
                                       "the update launched eagerly after each replay (timed by events)"
                               if res["graph"] else "every step launched eagerly"},
                "final_loss": res["loss"],
            })
            if "period_sweep" in res:
                out["period_sweep"] = {"workload": "BASELINE configs[2]: the headline step at each averaging period",
                                       "records": res["period_sweep"]}
            if "coda_round" in res:
                out["coda_round"] = res["coda_round"]
            if "training_eval" in res:
                out["training_eval"] = res["training_eval"]
        out["process_group"] = {"world_size": dist.get_world_size() if grouped() else 1,
                                "backend": dist.get_backend() if grouped() else None,
                                "rccl_version": ".".join(map(str, torch.cuda.nccl.version()))
                                if torch.cuda.is_available() and hasattr(torch.cuda, "nccl") else None,
                                "devices_visible": torch.cuda.device_count()}
        out["host"] = host
        out["gemm_selections"] = gemm_sel
        if sur is not None:
            out["surrogate_kernel"] = sur
        if r18 is not None:
            out["configs0"] = {"gpu": r18}
        if auc is not None:
            out["auc_eval"] = auc_record(auc, world, "configs[3]")
        if auc2 is not None:
            out["auc_eval_extreme"] = auc_record(auc2, world, "configs[4]")
        if cpu_baseline_on(args, world):
            threads = host["cpu_budget"]
            if res is not None:
                log("cpu baseline: resnet50 step")
                out["cpu_baseline"] = cpu_baseline_train_cores(args, host)
            if r18 is not None and args.cpu_workers > 0:
                log("cpu baseline: configs[0] gloo workers")
                c0 = cpu_baseline_configs0(args, host)
                more = all_cores_leg(host)
                if isinstance(more, int) and "value" in c0:
                    log(f"cpu baseline: configs[0] gloo workers on {more} threads (every usable CPU)")
                    c0["all_cores"] = cpu_baseline_configs0(args, host, threads_total=more, timeout=args.cpu_max_s * 2)
                elif not isinstance(more, int):
                    c0["all_cores"] = {"cores": host["affinity_cpus"], "skipped": more}
                out.setdefault("configs0", {})["cpu"] = c0
            torch.set_num_threads(threads)
            if auc is not None:
                log("cpu baseline: sklearn configs[3]")
                out["auc_eval"]["cpu_baseline"] = cpu_baseline_auc(auc)
            if auc2 is not None:
                log("cpu baseline: oracle + sklearn configs[4]")
                out["auc_eval_extreme"]["cpu_baseline"] = cpu_baseline_auc(
                    auc2, max_log2n=None if args.cpu_sklearn_full else 24, oracle_check=True)
        else:
            out["cpu_baseline"] = None
            if world > 1 and not args.no_cpu_baseline:
                out["cpu_baseline_note"] = ("timed at N = 1 only (the bench contract): the reference's CPU path "
                                            "does not depend on N, and rank 0's CPU minutes would hold every other "
                                            "rank at the closing barrier; see the N = 1 line")
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(_finite(out)) + "\n").encode())
    if grouped():
        dist.barrier(group=quiet)
        dist.destroy_process_group()


def _finite(x):
    """NaN / inf (an unmeasured figure) as null: the record stays strict JSON."""
    if isinstance(x, float):
        return x if math.isfinite(x) else None
    if isinstance(x, dict):
        return {k: _finite(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_finite(v) for v in x]
    return x


def load_profile(name: str, key: str):
    """One entry of a committed rocprofv3 PMC summary (profiles/<name>), or None."""
    f = REPO / "profiles" / name
    if not f.exists():
        return None
    try:
        rec = json.loads(f.read_text()).get(key)
    except Exception:
        return None
    if isinstance(rec, dict):
        rec = dict(rec, source=f"profiles/{name} (scripts/query_valu.py; rocprofv3 PMC + kernel trace, not this run)")
    return rec


def load_traffic(kernel: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    return load_profile("traffic.json", kernel)


if __name__ == "__main__":
    main()
