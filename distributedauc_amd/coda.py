"""CoDA: one rank's proximal primal-dual SGD with periodic model averaging.

Restates the training loop of main.py:83-339 on the flat HBM state
(flat.FlatState), with the hot path in HIP kernels:

  per step     label map + p_hat          1 launch  (dauc_label_map_phat)     main.py:303-310
               backbone forward           PyTorch-ROCm (MIOpen), bf16 autocast main.py:311
               surrogate loss + grads     1 launch  (dauc_surrogate_fwdbwd)   main.py:313-317, 326
               backbone backward          PyTorch-ROCm
               dppd_sg + running average  1 launch  (dauc_pd_update)          main.py:327, 333-334
  every I      all-reduce of flat[:n_reduce] over RCCL (params, a, b, alpha, class counts)
               + 1 launch (dauc_coda_finalize)                                main.py:292-301, 33-54
  per stage    alpha estimate: class sums (1 launch per batch), all-reduce,
               dauc_alpha_from_sums; anchor/average snapshots; stage-end divide main.py:144-208, 338-339

There is no host synchronisation inside a step (the reference syncs for p_hat
at main.py:309-310 every step). The reference's quirks are the
default (mode="reference"); mode="paper" applies the intended dual ascent.
"""
from __future__ import annotations

import contextlib
from typing import Callable, Iterator

import torch
import torch.distributed as dist
import torch.nn as nn

from . import ops
from .flat import FlatState
from .surrogate import auc_surrogate, auc_surrogate_logits, unit_seed


class CoDA:
    """CoDA state machine for one rank (main.py:83-339)."""

    def __init__(self, model: nn.Module, *, lr: float = 0.1, gamma: float = 2000.0, T0: int = 5000,
                 I: int = 2, split_index: int = 4, mode: str = "reference", world: int = 1, rank: int = 0,
                 group=None, autocast_dtype: torch.dtype | None = None, device=None,
                 max_exact_count: int = 1 << 24, head: str = "softmax", collective: bool | None = None,
                 weight_shadow: bool | None = None):
        if I < 1:
            raise ValueError("averaging period I must be >= 1")
        ops.mode_code(mode)  # validates
        if head not in ("softmax", "logits"):
            raise ValueError("head must be 'softmax' (model outputs probabilities, resnet.py:218) or 'logits'")
        self.head = head  # "logits": the model's softmax is folded into the surrogate kernel (§8f row 2)
        self.model = model
        self.state = FlatState(model, device)
        self.device = self.state.device
        self.lr0 = float(lr)
        self.gamma = float(gamma)
        self.T0 = int(T0)
        self.I = int(I)
        self.split_index = int(split_index)
        self.mode = mode
        self.world = int(world)
        self.rank = int(rank)
        self.group = group
        # collective: issue the averaging and alpha all-reduces (default: world > 1). True at world
        # 1 is the RCCL rehearsal: the world > 1 code path on a one-rank process group
        self.collective = self.world > 1 if collective is None else bool(collective)
        if collective and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("CoDA(collective=True) needs an initialised torch.distributed process group")
        self.autocast_dtype = autocast_dtype
        # bf16 autocast: the backbone's convolutions read their bf16 weights from one shadow buffer
        # cast once per forward (backbone.WeightShadow) instead of one cast launch per convolution
        if weight_shadow is None:
            weight_shadow = autocast_dtype == torch.bfloat16 and hasattr(model, "set_weight_shadow")
        if hasattr(model, "set_weight_shadow"):
            # always (re)set: this FlatState moved the parameters into a new buffer, so a shadow
            # left by an earlier CoDA / FlatState would mirror the old one
            model.set_weight_shadow(bool(weight_shadow))
        self.max_exact_count = max_exact_count
        self.t_total = 0
        self.stage = 0
        self.T = 0
        self.lr = self.lr0
        self.end_all = False
        self.t_in_stage = 0
        self._sums4 = torch.zeros(4, dtype=torch.float64, device=self.device)
        self._scratch = torch.zeros(8, dtype=torch.float32, device=self.device)
        self._ab_stage = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.last_loss: torch.Tensor | None = None
        self._graph_on = False
        self._graph_eager_update = False
        self._graph_grads = False  # p.grad holds a graph's static gradient buffers
        self._graph = None
        self._graph_key = None
        self.graph_captures = 0

    # ---------------------------------------------------------------- plumbing
    def _autocast(self):
        if self.autocast_dtype is None:
            return contextlib.nullcontext()
        return torch.autocast(device_type="cuda", dtype=self.autocast_dtype)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        with self._autocast():
            return self.model(x)

    def scores(self, x: torch.Tensor) -> torch.Tensor:
        """h = net(x)[:, 1] (resnet.py:218: column 1 of the softmax), fp32."""
        out = self.forward(x)
        if self.head == "logits":
            out = torch.softmax(out.float(), dim=1)
        h = out[:, 1]
        return h if h.dtype == torch.float32 else h.float()

    # ---------------------------------------------------------------- a6
    def average_all(self):
        """One CoDA round: main.py:40-54 (world > 1) / 297-299 (world == 1), then 300-301."""
        st = self.state
        if self.collective:
            dist.all_reduce(st.flat[: st.n_reduce], op=dist.ReduceOp.SUM, group=self.group)
        ops.coda_finalize(st.flat, st.n_avg, self.world, st.lcounts, st.gcounts)

    # ---------------------------------------------------------------- a7
    def begin_stage(self, s: int, batches: Iterator):
        """main.py:148-208: restart point, alpha estimate over 3**s batches, snapshots, T, lr."""
        st = self.state
        with torch.no_grad():
            if s > 1:
                st.params.copy_(st.avg)                 # main.py:149-150 (avg already / T)
                st.abalpha[:2].copy_(self._ab_stage)    # main.py:151-152
            self.model.eval()
            self._sums4.zero_()
            for _ in range(3 ** s):                     # main.py:172-188
                x, labels = next(batches)
                y8 = st.y8(labels.numel())
                self._scratch.zero_()
                ops.label_map_phat(labels, self.split_index, y8, self._scratch[0:2], self._scratch[2:4],
                                   self._scratch[4:5])
                if self.head == "logits":
                    ops.class_sums_logits(self.forward(x), y8, self._sums4, accumulate=True)
                else:
                    ops.class_sums(self.scores(x), y8, self._sums4, accumulate=True)
            self.model.train()
            if self.collective:
                dist.all_reduce(self._sums4, op=dist.ReduceOp.SUM, group=self.group)  # main.py:192-195
            ops.alpha_from_sums(self._sums4, st.alpha)  # main.py:197
            st.snapshot_anchor()                        # main.py:154 + 199-201
            self._ab_stage.copy_(st.abalpha[:2])        # a_average, b_average (main.py:207-208)
            st.reset_average()                          # main.py:206
        self.stage = s
        self.T = self.T0 * (3 ** (s - 1))               # main.py:202
        self.lr = self.lr0 * ((1 / 3) ** (s - 1))       # main.py:203

    def end_stage(self):
        """main.py:338-339: net_average /= T."""
        ops.scale_div(self.state.avg, float(self.T))

    # ---------------------------------------------------------------- a1-a5
    def train_step(self, x: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """main.py:289-334 for one batch already on the device. Returns the loss (device scalar)."""
        st = self.state
        B = labels.numel()
        if self.world * self.I * B >= self.max_exact_count:
            raise ValueError("world*I*batch must stay below 2^24 so the fp32 count slots stay exact")
        self.t_total += 1
        if self.t_total % self.I == 0:
            with torch.no_grad():
                self.average_all()
        self.last_loss = self._graphed_body(x, labels) if self._graph_on else self.step_body(x, labels)
        return self.last_loss

    def step_body(self, x: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """main.py:303-334 without the round trigger: label map + p_hat, forward, surrogate,
        backward, pd_update, zero_grad. Stream-ordered with no host sync, so it can be
        captured in a HIP graph (the lr it bakes in changes only at a stage start)."""
        if self._graph_grads:  # leave graph mode: the next backward must not add into its buffers
            self.model.zero_grad(set_to_none=True)
            self._graph_grads = False
        loss = self._forward_backward(x, labels)
        self.state.update(self.lr, self.gamma, self.mode)
        self.model.zero_grad(set_to_none=True)
        return loss

    def _forward_backward(self, x: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """main.py:303-326: label map + p_hat, forward, surrogate, backward (gradients in p.grad)."""
        st = self.state
        y8 = st.y8(labels.numel())
        ops.label_map_phat(labels, self.split_index, y8, st.lcounts, st.gcounts, st.p_hat)
        if self.head == "logits":
            loss = auc_surrogate_logits(self.forward(x), y8, st.abalpha, st.p_hat, st.grad3)
        else:
            loss = auc_surrogate(self.scores(x), y8, st.abalpha, st.p_hat, st.grad3)
        loss.backward(unit_seed(loss.device))  # no ones_like fill, no dF/dh * 1 pass
        return loss.detach()

    # ---------------------------------------------------------------- HIP graph replay
    def use_graph(self, enable: bool = True, eager_update: bool = False) -> "CoDA":
        """Replay step_body (label map, forward, surrogate, backward, pd_update, zero_grad) as ONE
        HIP graph: a small batch's step is bound by the ~200 kernel launches of the backbone, not
        by the GPU. The averaging round stays outside the graph (RCCL, every I steps), so the
        schedule is the reference's. The graph is captured at the first step of each (input
        shape, dtype, lr) — lr changes only at a stage start — after two warm-up bodies on a
        side stream whose effect on the state is undone; every replay reads the batch from the
        graph's own input buffers, so the caller's tensors are copied in first.

        ``eager_update``: the graph holds label map -> forward -> surrogate -> backward only, and
        the update (dppd_sg + running average, ONE launch) runs eagerly after each replay from
        the gradients the replay left in the parameters' (static) .grad buffers. The update is
        then an ordinary launch on the stream -- timed by events like in eager mode -- and lr is
        not baked into the graph (no re-capture at a stage start)."""
        self._graph_on = bool(enable)
        self._graph_eager_update = bool(enable and eager_update)
        self._graph = self._graph_key = None
        if self._graph_grads:
            self.model.zero_grad(set_to_none=True)
            self._graph_grads = False
        return self

    def _graphed_body(self, x: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        key = (tuple(x.shape), x.dtype, x.stride(), tuple(labels.shape), labels.dtype,
               None if self._graph_eager_update else self.lr)
        if self._graph is None or self._graph_key != key:
            self._capture(x, labels, key)
        self._gx.copy_(x)
        self._gy.copy_(labels)
        self._graph.replay()
        if self._graph_eager_update:
            self.state.update(self.lr, self.gamma, self.mode)  # reads the replay's static .grad buffers
        # the graph's loss buffer is overwritten by the next replay: hand out a copy, as eager does
        return self._gloss.clone()

    def _capture(self, x: torch.Tensor, labels: torch.Tensor, key) -> None:
        st = self.state
        state = [st.flat, st.avg, st.lcounts, st.gcounts, st.p_hat, *self.model.buffers()]
        self._graph = None
        with torch.no_grad():
            snap = [t.clone() for t in state]
            self._gx, self._gy = x.clone(), labels.clone()
        cur = torch.cuda.current_stream(self.device)
        side = torch.cuda.Stream(self.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(2):  # lazy initialisation (engine choices, workspaces) before capture
                self.step_body(self._gx, self._gy)
        cur.wait_stream(side)
        with torch.no_grad():
            for t, s in zip(state, snap):
                t.copy_(s)
        graph = torch.cuda.CUDAGraph()
        # thread_local: a communicator's helper threads (RCCL's proxy) may touch the runtime while
        # this thread captures; only this thread's calls must be capturable
        if self._graph_grads:
            self.model.zero_grad(set_to_none=True)
            self._graph_grads = False
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            if self._graph_eager_update:
                # the backward's gradient tensors become p.grad (static: every replay rewrites them)
                self._gloss = self._forward_backward(self._gx, self._gy)
            else:
                self._gloss = self.step_body(self._gx, self._gy)
        self._graph_grads = self._graph_eager_update
        self._graph, self._graph_key = graph, key
        self.graph_captures += 1

    # ---------------------------------------------------------------- loop
    def run(self, batches: Iterator, *, num_stages: int, total_iter: int, test_freq: int | None = None,
            evaluate: Callable[["CoDA"], None] | None = None,
            on_step: Callable[["CoDA"], None] | None = None,
            checkpoint_every: int | None = None, checkpoint_path: str | None = None):
        """The full schedule of main.py:140-339 (stages 1 .. num_stages-1).

        ``on_step`` (optional) is called after every training step (history, tests).
        A CoDA restored with ``load()`` resumes at the saved stage and step (the caller
        resumes its batch stream); ``checkpoint_every`` saves every that many steps.
        """
        resuming = self.stage > 0
        if not resuming:
            with torch.no_grad():
                self.average_all()  # main.py:141-142
        first = self.stage if resuming else 1
        for s in range(first, num_stages):
            if self.end_all:
                break
            if resuming and s == first:
                start = self.t_in_stage
            else:
                self.begin_stage(s, batches)
                start = 0
            for t in range(start, self.T):
                self.t_in_stage = t
                if test_freq and evaluate is not None and self.t_total % test_freq == 0:
                    evaluate(self)  # main.py:215-270
                if self.t_total > total_iter:  # main.py:273-275
                    self.end_all = True
                    break
                x, labels = next(batches)
                self.train_step(x, labels)
                self.t_in_stage = t + 1
                if on_step is not None:
                    on_step(self)
                if checkpoint_every and checkpoint_path and self.t_total % checkpoint_every == 0:
                    self.save(checkpoint_path)
            self.end_stage()
            self.t_in_stage = self.T

    # ---------------------------------------------------------------- checkpoint / resume
    def state_dict(self) -> dict:
        """Everything a resumed run needs (the reference has no checkpointing)."""
        st = self.state
        return {
            "flat": st.flat.detach().clone(), "anchor": st.anchor.clone(), "avg": st.avg.clone(),
            "gcounts": st.gcounts.clone(), "p_hat": st.p_hat.clone(), "ab_stage": self._ab_stage.clone(),
            "buffers": {n: b.detach().clone() for n, b in self.model.named_buffers()},
            "counters": torch.tensor([self.t_total, self.stage, self.T, self.t_in_stage, int(self.end_all)],
                                     dtype=torch.int64),
            "lr": torch.tensor([self.lr], dtype=torch.float64),
            "layout": torch.tensor([e[2] for e in st.entries] + [st.n_params], dtype=torch.int64),
        }

    def load_state_dict(self, sd: dict) -> None:
        st = self.state
        layout = torch.tensor([e[2] for e in st.entries] + [st.n_params], dtype=torch.int64)
        if not torch.equal(sd["layout"].cpu(), layout):
            raise ValueError("checkpoint was written for a different model layout")
        with torch.no_grad():
            st.flat.copy_(sd["flat"])
            st.anchor.copy_(sd["anchor"])
            st.avg.copy_(sd["avg"])
            st.gcounts.copy_(sd["gcounts"])
            st.p_hat.copy_(sd["p_hat"])
            self._ab_stage.copy_(sd["ab_stage"])
            bufs = dict(self.model.named_buffers())
            for n, b in sd["buffers"].items():
                bufs[n].copy_(b)
        self.t_total, self.stage, self.T, self.t_in_stage, end_all = (int(v) for v in sd["counters"].tolist())
        self.end_all = bool(end_all)
        self.lr = float(sd["lr"][0])

    def save(self, path: str) -> None:
        import os

        tmp = f"{path}.tmp"
        torch.save(self.state_dict(), tmp)
        os.replace(tmp, path)

    def load(self, path: str) -> None:
        self.load_state_dict(torch.load(path, map_location=self.device, weights_only=True))

    def stage_lengths(self, num_stages: int) -> list[int]:
        return [self.T0 * 3 ** (s - 1) for s in range(1, num_stages)]

    @staticmethod
    def p_prior(split_index: int, neg_keep_ratio: float, num_classes: int = 1000) -> float:
        """main.py:86-87: the positive prior used only for the run label."""
        p_pos = (split_index + 1.0) / num_classes
        return p_pos / (p_pos + (1 - p_pos) * neg_keep_ratio)

    def __repr__(self):
        n = self.state.numel()
        return (f"CoDA(params={n}, I={self.I}, T0={self.T0}, lr0={self.lr0}, gamma={self.gamma}, "
                f"mode={self.mode}, world={self.world}, rank={self.rank}, collective={self.collective}, "
                f"flat_MB={4 * n / 2**20:.1f})")

