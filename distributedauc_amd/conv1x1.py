"""Stride-1 1x1 convolutions of the channels-last backbone as plain GEMMs where that is faster.

In NHWC a 1x1 convolution is a GEMM over the [M, C] view of the activation (M = N*H*W):
    forward  y[M, Cout]     = x[M, Cin] @ W[Cout, Cin]^T
    dgrad    dx[M, Cin]     = dy[M, Cout] @ W
    wgrad    dW[Cout, Cin]  = dy^T @ x   (K = M: split over S slabs, fp32 partial sums)
MIOpen's implicit-GEMM convolutions zero their output before every launch and lose to hipBLASLt
on most ResNet-50 1x1 shapes (profiles/r01/probe_conv1x1.log), but not on all of them (the
large-M / small-C layer1 shapes favour MIOpen). So each (shape, direction) is timed once, on
first use, with both engines on the live stream (HIP events, best of 3) and the faster one is
kept - the cudnn.benchmark idea, per direction. Numerics: bf16 operands, fp32 accumulation,
bf16 activations / fp32 weight gradient (the fp32 master weight's grad is returned directly,
so autocast's cast-back kernel disappears too).
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .ops import _ptr, _stream, check, strided_add_, strided_pick

__all__ = ["conv1x1", "conv1x1_skip", "Conv1x1Function", "Conv1x1SkipFunction", "plans", "dump_plans"]

plans: dict = {}  # (M, Cin, Cout, dtype, direction) -> engine

# Engine choices measured once on MI355X for the bench shapes (ResNet-50 b256 and ResNet-18 b32,
# 224^2, bf16 channels-last; scripts/gpu_conv1x1_plans.sh): shapes listed here are never timed at
# run time, so every rank (and every run) uses the same engines and the same numerics. Shapes
# not listed are timed on first use; DAUC_CONV1X1_PLANS names another file ("" = none).
# the strided downsample's backward: "gemm" (GEMMs on x[:, :, ::s, ::s]) or "miopen" (one
# convolution_backward call; kept as the A/B reference, DAUC_DOWNSAMPLE_BWD=miopen)
_DOWNSAMPLE_BWD = os.environ.get("DAUC_DOWNSAMPLE_BWD", "gemm")
PLANS_FILE = os.environ.get("DAUC_CONV1X1_PLANS", os.path.join(os.path.dirname(__file__), "conv1x1_plans.json"))


def _plan_key(key) -> str:
    M, cin, cout, dtype, direction = key
    return f"{M},{cin},{cout},{str(dtype).replace('torch.', '')},{direction}"


def _arch() -> str:
    """gcnArchName of the current device without its feature suffixes (e.g. "gfx950")."""
    return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]


def _load_plans() -> None:
    if not PLANS_FILE or not os.path.exists(PLANS_FILE):
        return
    import json

    dtypes = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32}
    with open(PLANS_FILE) as f:
        doc = json.load(f)
    # the plan was measured on one GPU architecture: on any other the engines are timed again
    if doc.get("arch") and torch.cuda.is_available() and doc["arch"] != _arch():
        return
    for k, eng in doc.get("plans", {}).items():
        M, cin, cout, dt, direction = k.split(",")
        plans.setdefault((int(M), int(cin), int(cout), dtypes[dt], direction), eng)


def dump_plans(path: str) -> None:
    """Write the engine choice of every (shape, direction) seen so far (the shipped plan file's format)."""
    import json

    with open(path, "w") as f:
        json.dump({"device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else None,
                   "arch": _arch() if torch.cuda.is_available() else None,
                   "plans": {_plan_key(k): v for k, v in sorted(plans.items(), key=lambda kv: _plan_key(kv[0]))}},
                  f, indent=1)



def _timed(fn, reps=3):
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best


_FORCE = os.environ.get("DAUC_CONV1X1", "auto")  # auto | gemm | conv (fixed engine: reproducible runs)
_loaded: list = []
_fixed: list = []  # fixed_engine() stack


@contextlib.contextmanager
def fixed_engine(name: str = "gemm"):
    """Inside: every 1x1 convolution runs on engine `name` (gemm | conv), untimed and ignoring the
    plans. For results that must not depend on a timing: the split evaluation scores the test set
    on every rank and needs the same bits as one rank scoring it all (main.Evaluator)."""
    _fixed.append(name)
    try:
        yield
    finally:
        _fixed.pop()


def _choose(key, candidates: dict):
    if _fixed:
        eng = next((n for n in candidates if n.startswith(_fixed[-1])), None)
        if eng == "gemm8" and "gemm32" in candidates:
            eng = "gemm32"
        if eng is not None:
            return eng
    if not _loaded:
        _load_plans()
        _loaded.append(True)
    # a forced engine (DAUC_CONV1X1=gemm|conv) wins over the shipped plan
    eng = plans.get(key) if _FORCE == "auto" else None
    if eng is None and _FORCE != "auto":
        eng = next((n for n in candidates if n.startswith(_FORCE)), None)
        if eng == "gemm8" and "gemm32" in candidates:
            eng = "gemm32"
        if eng is not None:
            plans[key] = eng
    if eng is None:
        times = {name: _timed(fn) for name, fn in candidates.items()}
        eng = min(times, key=times.get)
        plans[key] = eng
    return eng


def _wgrad_gemm(g2, x2, slabs):
    M, cout = g2.shape
    cin = x2.shape[1]
    if slabs == 1:
        return torch.mm(g2.t(), x2, out_dtype=torch.float32)
    part = torch.bmm(g2.view(slabs, M // slabs, cout).transpose(1, 2), x2.view(slabs, M // slabs, cin),
                     out_dtype=torch.float32)
    if (cout * cin) % 4:
        return part.sum(0)
    out = torch.empty((cout, cin), dtype=torch.float32, device=part.device)
    check(_lib.load().dauc_slab_sum(_ptr(part), slabs, cout * cin, _ptr(out), _stream(part.device)),
          "dauc_slab_sum")
    return out


def _low(weight, dtype):
    """The weight in the activations' dtype: the backbone's bf16 shadow when one is live (one cast
    launch per forward for every conv), else a cast of its own."""
    from .backbone import shadow_weight

    wb = shadow_weight(weight, dtype)
    return wb.detach() if wb is not None else weight.detach().to(dtype)


def _fwd(x, weight):
    """y = conv1x1(x, weight) (bf16 operands as x, fp32 accumulation), engine timed per shape."""
    N, cin, H, W = x.shape
    cout = weight.shape[0]
    M = N * H * W
    wc = _low(weight, x.dtype).reshape(cout, cin)
    x2 = x.permute(0, 2, 3, 1).reshape(M, cin)  # a view: x is channels-last contiguous
    with torch.autocast("cuda", enabled=False):
        key = (M, cin, cout, x.dtype, "fwd")
        eng = _choose(key, {"gemm": lambda: torch.mm(x2, wc.t()),
                            "conv": lambda: F.conv2d(x, wc.view(cout, cin, 1, 1))})
        if eng == "gemm":
            y = torch.mm(x2, wc.t()).view(N, H, W, cout).permute(0, 3, 1, 2)
        else:
            y = F.conv2d(x, wc.view(cout, cin, 1, 1)).contiguous(memory_format=torch.channels_last)
    return y, wc


def _prep_grad(gy, x, cout):
    N, cin, H, W = x.shape
    gy = gy.to(x.dtype).contiguous(memory_format=torch.channels_last)
    return gy, gy.permute(0, 2, 3, 1).reshape(N * H * W, cout)


def _conv_dgrad(gy, x, wc):
    cout, cin = wc.shape
    return torch.ops.aten.convolution_backward(gy, x, wc.view(cout, cin, 1, 1), None, [1, 1], [0, 0], [1, 1],
                                               False, [0, 0], 1, [True, False, False])[0]


def _fconv_dgrad(gy, wc):
    """dx = dy @ W as a FORWARD 1x1 convolution of dy with W^T (C_in' = cout, C_out' = cin): the
    forward solvers (CK, no output zero-fill) instead of MIOpen's backward-data kernel, which zeroes
    its output first (ResNet-50 layer1 256 -> 64: 102 + 25 us against a ~42 us forward)."""
    cout, cin = wc.shape
    return F.conv2d(gy, wc.t().contiguous().view(cin, cout, 1, 1)).contiguous(memory_format=torch.channels_last)


def _dgrad(gy, g2, x, wc):
    """dx = dy @ W (a new channels-last tensor)."""
    N, cin, H, W = x.shape
    cout = wc.shape[0]
    M = N * H * W
    with torch.autocast("cuda", enabled=False):
        eng = _choose((M, cin, cout, x.dtype, "dgrad"),
                      {"gemm": lambda: torch.mm(g2, wc), "conv": lambda: _conv_dgrad(gy, x, wc),
                       "fconv": lambda: _fconv_dgrad(gy, wc)})
        if eng == "gemm":
            return torch.mm(g2, wc).view(N, H, W, cin).permute(0, 3, 1, 2)
        if eng == "fconv":
            return _fconv_dgrad(gy, wc)
        return _conv_dgrad(gy, x, wc).contiguous(memory_format=torch.channels_last)


def _dgrad_acc(base, gy, g2, x, wc):
    """base += dy @ W in place (base: a channels-last tensor shaped like x that this backward owns).
    GEMM engine: one launch with beta = 1 (reads base once, writes it once, one rounding), instead
    of a dgrad output plus autograd's separate add pass (read 2, write 1). C aliases D here; on
    MI355X every engine / tuned solution of these shapes returns the same bits for the aliased
    in-place form as for the out-of-place one (profiles/r02/tunableop/tunableop_probe.jsonl), and
    out-of-place torch.addmm would first copy C into D (2 x 411 MB more traffic at layer 1)."""
    N, cin, H, W = x.shape
    cout = wc.shape[0]
    M = N * H * W
    b2 = base.permute(0, 2, 3, 1).reshape(M, cin)  # a view of base
    with torch.autocast("cuda", enabled=False):
        key = (M, cin, cout, x.dtype, "dgrad_acc")
        if not _loaded:
            _load_plans()
            _loaded.append(True)
        eng = None if _fixed else plans.get(key)
        if eng is None and _fixed:
            eng = _choose(key, {"gemm": None, "conv": None, "fconv": None})  # fixed_engine(): never timed
        elif eng is None:
            scratch = base.clone(memory_format=torch.channels_last)
            s2 = scratch.permute(0, 2, 3, 1).reshape(M, cin)
            eng = _choose(key, {"gemm": lambda: s2.addmm_(g2, wc),
                                "conv": lambda: scratch.add_(_conv_dgrad(gy, x, wc)),
                                "fconv": lambda: scratch.add_(_fconv_dgrad(gy, wc))})
            del scratch, s2
        if eng == "gemm":
            b2.addmm_(g2, wc)
        elif eng == "fconv":
            base.add_(_fconv_dgrad(gy, wc))
        else:
            base.add_(_conv_dgrad(gy, x, wc))
    return base


def _wgrad(gy, g2, x, wc, wdtype):
    N, cin, H, W = x.shape
    cout = wc.shape[0]
    M = N * H * W
    x2 = x.permute(0, 2, 3, 1).reshape(M, cin)
    with torch.autocast("cuda", enabled=False):
        def conv_w():
            return torch.ops.aten.convolution_backward(gy, x, wc.view(cout, cin, 1, 1), None, [1, 1], [0, 0], [1, 1],
                                                       False, [0, 0], 1, [False, True, False])[1]

        cands = {"conv": conv_w}
        for s in (8, 32, 128):
            if M % s == 0 and M // s >= 64:
                cands[f"gemm{s}"] = (lambda s=s: _wgrad_gemm(g2, x2, s))
        eng = _choose((M, cin, cout, x.dtype, "wgrad"), cands)
        if eng == "conv":
            dw = conv_w().reshape(cout, cin).to(wdtype)
        else:
            dw = _wgrad_gemm(g2, x2, int(eng[4:])).to(wdtype)
    return dw.view(cout, cin, 1, 1)


def _cl_ok(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 4 and t.shape[1] % 8 == 0
            and t.is_contiguous(memory_format=torch.channels_last) and t.data_ptr() % 16 == 0)


def _pick(x: torch.Tensor, s: int) -> torch.Tensor:
    """x[:, :, ::s, ::s] as a channels-last tensor (csrc/strided.hip at HBM rate; torch's strided copy
    ran at 2.9 TB/s)."""
    if _cl_ok(x):
        return strided_pick(x, s)
    return x[:, :, ::s, ::s].contiguous(memory_format=torch.channels_last)


def _add_strided(dx: torch.Tensor, src: torch.Tensor, s: int) -> None:
    """dx[:, :, ::s, ::s] += src (csrc/strided.hip; the bits of torch's add_)."""
    if _cl_ok(dx) and _cl_ok(src):
        strided_add_(dx, src, s)
    else:
        dx[:, :, ::s, ::s].add_(src)


class Conv1x1Function(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        y, wc = _fwd(x, weight)
        ctx.save_for_backward(x, wc)
        ctx.wdtype = weight.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wc = ctx.saved_tensors
        gy, g2 = _prep_grad(gy, x, wc.shape[0])
        dx = _dgrad(gy, g2, x, wc) if ctx.needs_input_grad[0] else None
        dw = _wgrad(gy, g2, x, wc, ctx.wdtype) if ctx.needs_input_grad[1] else None
        return dx, dw


class Conv1x1SkipFunction(torch.autograd.Function):
    """(conv1(x), skip) for a bottleneck block's input x: skip = x (identity) or the 1x1 downsample
    conv of x (resnet.py:87-108; stride 1 as a GEMM, stride 2 forward through MIOpen). Backward:
    dx = d(skip) + dgrad(conv1), the conv1 dgrad GEMM accumulating into the skip term in place
    (beta = 1), so the branch-point gradient sum that autograd would run as a separate add kernel
    over the block input (ResNet-50 b256: up to 3 x 411 MB per block) disappears.

    The strided downsample's backward runs as GEMMs on xs = x[:, :, ::s, ::s] (one strided copy of a
    quarter of x): dWd = dy^T xs (the split-K fp32 engine) and dxs = dy Wd, added at the strided
    positions of the conv1 dgrad's output. MIOpen's backward-data zero-fills the whole input
    gradient and its backward-weights a workspace, then casts (ResNet-50 b256 layer2.0: ~105 us +
    fill, ~120 us + fill + cast). Its forward stays on the convolution solvers, which beat the
    strided copy + GEMM (profiles/r05/downsample_gemm/)."""

    @staticmethod
    def forward(ctx, x, w1, wd, skip_grad_owned, down_stride=1):
        y1, wc1 = _fwd(x, w1)
        ctx.down_stride = int(down_stride)
        if wd is None:
            skip, wcd = x, None
        elif down_stride == 1:
            skip, wcd = _fwd(x, wd)
        else:
            wcd = _low(wd, x.dtype).reshape(wd.shape[0], wd.shape[1])
            with torch.autocast("cuda", enabled=False):
                skip = F.conv2d(x, wcd.view(*wd.shape), stride=down_stride).contiguous(
                    memory_format=torch.channels_last)
        ctx.save_for_backward(x, wc1, wcd)
        ctx.wdtypes = (w1.dtype, None if wd is None else wd.dtype)
        ctx.skip_grad_owned = bool(skip_grad_owned)
        return y1, skip

    @staticmethod
    def backward(ctx, g1, gs):
        x, wc1, wcd = ctx.saved_tensors
        dx = dw1 = dwd = None
        gy1 = g21 = gyd = g2d = None
        if g1 is not None:
            gy1, g21 = _prep_grad(g1, x, wc1.shape[0])
        strided = wcd is not None and ctx.down_stride != 1
        s = ctx.down_stride
        xd = x  # the downsample GEMMs' input
        dx_down = dwd_s = None
        if gs is not None and strided and _DOWNSAMPLE_BWD == "miopen":  # A/B reference only
            gsd = gs.to(x.dtype).contiguous(memory_format=torch.channels_last)
            cout, cin = wcd.shape
            with torch.autocast("cuda", enabled=False):
                dx_down, dwd_s, _ = torch.ops.aten.convolution_backward(
                    gsd, x, wcd.view(cout, cin, 1, 1), None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                    [bool(ctx.needs_input_grad[0]), bool(ctx.needs_input_grad[2]), False])
        elif gs is not None and wcd is not None:
            if strided:
                xd = _pick(x, s)
            gyd, g2d = _prep_grad(gs, xd, wcd.shape[0])
        if ctx.needs_input_grad[0]:
            if gs is None:
                base = None
            elif wcd is None:
                # the identity branch's gradient. With the fused BN node as its consumer it is a
                # fresh tensor (BnActFunction's dres) seen only here, so it is accumulated into in
                # place; otherwise (e.g. torch's add, which hands one tensor to both operands) a copy
                base = gs.to(x.dtype).contiguous(memory_format=torch.channels_last)
                if base is gs and not ctx.skip_grad_owned:
                    base = base.clone(memory_format=torch.channels_last)
            elif strided:
                base = None if dx_down is None else dx_down.contiguous(memory_format=torch.channels_last)
            else:
                base = _dgrad(gyd, g2d, x, wcd)
            if g1 is None:
                dx = base
            elif base is None:
                dx = _dgrad(gy1, g21, x, wc1)
            else:
                dx = _dgrad_acc(base, gy1, g21, x, wc1)
            if strided and gs is not None and dx_down is None:
                if dx is None:
                    dx = torch.zeros_like(x, memory_format=torch.channels_last)
                _add_strided(dx, _dgrad(gyd, g2d, xd, wcd), s)
        if ctx.needs_input_grad[1] and g1 is not None:
            dw1 = _wgrad(gy1, g21, x, wc1, ctx.wdtypes[0])
        if wcd is not None and ctx.needs_input_grad[2] and gs is not None:
            if dwd_s is not None:
                dwd = dwd_s.to(ctx.wdtypes[1]).view(wcd.shape[0], wcd.shape[1], 1, 1)
            else:
                dwd = _wgrad(gyd, g2d, xd, wcd, ctx.wdtypes[1])
        return dx, dw1, dwd, None, None


def conv1x1(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """``conv(x)`` for a bias-free, stride-1, ungrouped 1x1 conv on a channels-last GPU tensor;
    anything else goes to the module itself."""
    if (conv.kernel_size != (1, 1) or conv.stride != (1, 1) or conv.groups != 1 or conv.bias is not None
            or conv.padding != (0, 0) or x.device.type != "cuda"
            or not x.is_contiguous(memory_format=torch.channels_last)):
        return conv(x)
    if torch.is_autocast_enabled("cuda") and x.dtype == torch.float32:
        x = x.to(torch.get_autocast_dtype("cuda"))
    return Conv1x1Function.apply(x, conv.weight)


def _gemm_ok(conv: nn.Conv2d | None, x: torch.Tensor, any_stride: bool = False) -> bool:
    return conv is None or (conv.kernel_size == (1, 1) and conv.groups == 1 and conv.bias is None
                            and conv.padding == (0, 0) and conv.dilation == (1, 1)
                            and (conv.stride == (1, 1) or (any_stride and conv.stride[0] == conv.stride[1])))


def conv1x1_skip(conv: nn.Conv2d, x: torch.Tensor, down: nn.Conv2d | None = None, skip_grad_owned: bool = False):
    """``(conv(x), x if down is None else down(x))`` for a bottleneck's stride-1 1x1 conv1 and its
    identity / 1x1 downsample branch (any stride), with the branch-point gradient sum fused into the
    dgrad GEMM (Conv1x1SkipFunction). ``skip_grad_owned``: the skip's consumer hands back a gradient
    tensor nobody else holds (the fused BN node does), so it may be accumulated into in place.
    Other shapes: the two branches separately."""
    if (x.device.type != "cuda" or not x.is_contiguous(memory_format=torch.channels_last)
            or not _gemm_ok(conv, x) or not _gemm_ok(down, x, any_stride=True)):
        return conv1x1(conv, x), (x if down is None else conv1x1(down, x))
    if torch.is_autocast_enabled("cuda") and x.dtype == torch.float32:
        x = x.to(torch.get_autocast_dtype("cuda"))
    return Conv1x1SkipFunction.apply(x, conv.weight, None if down is None else down.weight, skip_grad_owned,
                                     1 if down is None else down.stride[0])
