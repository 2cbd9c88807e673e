"""The two-step sharded exact AUC at the BASELINE sizes, against the C oracle.

dauc_auc_eval_compact_part -> (the all-gather, simulated by copying the G slots side by side) ->
dauc_auc_eval_query_part for every part, at configs[3] (2^24 scores, 1 % positives, G = 2, 4, 8)
and configs[4] (2^27, 0.1 %, G = 8) drawn by the bench's own generator: the parts' (W, T) sum to
the oracle's integers, every record carries the oracle's P and a zero consistency word. The
verdict-2 routes at full size: an unshuffled 2^24 test set (every positive in slice 0, which
overflows its slot) and tables past the count index's capacity with no slot overflowing (ADVICE
r04) -- every part reports verdict 2 and the blocking sorted path gives the oracle's integers. Then
ExactAUC itself through 2 real gloo ranks on cuda:0 at 2^24 (the sharded path with its two
all-gathers), with the cross-rank checks: labels or lengths that differ between the ranks raise on
both. Reference: main.py:79-81, 232-250; sklearn _ranking.py:826-908."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch

from oracle import coracle

pytestmark = pytest.mark.gpu


def _two_step(dev, ts, ty, G):
    from distributedauc_amd import ops

    n = ts.numel()
    nb = ops.auc_slot_bytes(n, G)
    slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
    for r in range(G):
        ops.auc_eval_compact_part(ts, ty, r, G, slots[r * nb:(r + 1) * nb])
    return [_query(dev, ts, ty, r, G, slots) for r in range(G)]


def _query(dev, ts, ty, r, G, slots, out=None):
    """Rank r's step 2 as a rank runs it: its own step 1 just before (the G simulated ranks share
    one workspace here, and step 2 consumes the build state step 1 prepares there)."""
    from distributedauc_amd import ops

    nb = ops.auc_slot_bytes(ts.numel(), G)
    ops.auc_eval_compact_part(ts, ty, r, G, torch.empty(nb, dtype=torch.uint8, device=dev))
    return ops.auc_eval_query_part(ts, ty, r, G, slots, out=out).cpu().tolist()


def _sorted_parts(dev, ts, ty, G):
    from distributedauc_amd import ops

    W = Tt = 0
    for r in range(G):
        o = ops.auc_eval_counts_part(ts, ty, r, G, torch.zeros(3, dtype=torch.int64, device=dev))
        W, Tt = W + o[0], Tt + o[1]
    return W, Tt


def _oracle(ts, ty):
    return coracle.auc_counts(ty.cpu().numpy().astype(np.int64), ts.cpu().numpy())


@pytest.mark.timeout(300)
def test_two_step_configs3_sizes(dev):
    """configs[3]: 2^24 fp32 scores at 1 % positives, G = 2, 4, 8: bit-exact vs the C oracle."""
    from distributedauc_amd.loader import synthetic_scores

    ts, ty = synthetic_scores(1 << 24, 0.01, dev)
    e = _oracle(ts, ty)
    for G in (2, 4, 8):
        recs = _two_step(dev, ts, ty, G)
        assert {(v[3], v[4], v[5], v[6], v[7]) for v in recs} == {(e["P"], 0, 0, 0, 1)}, (G, recs)
        assert sum(v[2] for v in recs) == 0
        assert (sum(v[0] for v in recs), sum(v[1] for v in recs)) == (e["wins"], e["ties"]), G


@pytest.mark.timeout(300)
def test_two_step_configs4_size(dev):
    """configs[4]: 2^27 fp32 scores at 0.1 % positives, G = 8: bit-exact vs the C oracle."""
    from distributedauc_amd.loader import synthetic_scores

    ts, ty = synthetic_scores(1 << 27, 0.001, dev)
    e = _oracle(ts, ty)
    recs = _two_step(dev, ts, ty, 8)
    assert {(v[3], v[4], v[5], v[6], v[7]) for v in recs} == {(e["P"], 0, 0, 0, 1)}, recs
    assert (sum(v[0] for v in recs), sum(v[1] for v in recs)) == (e["wins"], e["ties"])


@pytest.mark.timeout(300)
def test_two_step_unshuffled_overflow_2e24(dev):
    """An unshuffled 2^24 test set: the 1 % positives all sit in slice 0, far past its slot's
    capacity -- every part reports verdict 2 (and a zero check word), and the blocking sorted path
    over the parts gives the oracle's integers."""
    from distributedauc_amd import ops
    from distributedauc_amd.loader import synthetic_scores

    ts, _ = synthetic_scores(1 << 24, 0.01, dev)
    P = (1 << 24) // 100
    ty = torch.where(torch.arange(1 << 24, device=dev) < P, 1, -1).to(torch.int8)
    e = _oracle(ts, ty)
    G = 8
    assert P > ops.auc_slot_bytes(1 << 24, G) // 4  # slice 0 cannot hold them
    recs = _two_step(dev, ts, ty, G)
    assert {(v[3], v[4], v[7]) for v in recs} == {(e["P"], 0, 2)}, recs
    assert _sorted_parts(dev, ts, ty, G) == (e["wins"], e["ties"])


def _gathered(dev, ts, ty, G):
    """The G slots side by side (the all-gather) and every part's step-2 record."""
    from distributedauc_amd import ops

    n = ts.numel()
    nb = ops.auc_slot_bytes(n, G)
    slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
    for r in range(G):
        ops.auc_eval_compact_part(ts, ty, r, G, slots[r * nb:(r + 1) * nb])
    return slots, [_query(dev, ts, ty, r, G, slots) for r in range(G)]


def _sorted_fallback(dev, ts, ty, G, slots, P):
    """Every part's dauc_auc_eval_query_part_sorted record."""
    from distributedauc_amd import ops

    return [ops.auc_eval_query_part_sorted(ts, ty, r, G, slots, P).cpu().tolist() for r in range(G)]


@pytest.mark.parametrize("G", [2, 8])
@pytest.mark.timeout(300)
def test_two_step_sorted_fallback_tie_heavy(dev, G):
    """configs[3]'s scores rounded to bf16 (1,377 distinct positive values: the slotted index
    refuses the table, verdict 2 on every part): dauc_auc_eval_query_part_sorted sorts the gathered
    slots' positives and counts each part's own slice through the distinct-key index -- verdict 1
    everywhere, the parts' (W, T) sum to the oracle's, no whole-vector compaction."""
    from distributedauc_amd.loader import synthetic_scores

    ts, ty = synthetic_scores(1 << 24, 0.01, dev)
    ts = ts.bfloat16().float()
    e = _oracle(ts, ty)
    slots, recs = _gathered(dev, ts, ty, G)
    assert {(v[3], v[7]) for v in recs} == {(e["P"], 2)}, recs
    got = _sorted_fallback(dev, ts, ty, G, slots, e["P"])
    assert {(v[2], v[3], v[7]) for v in got} == {(0, e["P"], 1)}, got
    assert (sum(v[0] for v in got), sum(v[1] for v in got)) == (e["wins"], e["ties"])


@pytest.mark.timeout(300)
def test_two_step_sorted_fallback_refuses_what_slots_cannot_serve(dev):
    """The sorted two-step fallback reports verdict 2 (the caller's whole-vector path) when a slot
    overflowed (an unshuffled test set), when P exceeds the slots' total, and when the positives are
    the larger class."""
    from distributedauc_amd.loader import synthetic_scores

    G = 8
    ts, _ = synthetic_scores(1 << 22, 0.01, dev)
    P = (1 << 22) // 20
    ty = torch.where(torch.arange(1 << 22, device=dev) < P, 1, -1).to(torch.int8)
    slots, _ = _gathered(dev, ts, ty, G)
    assert {v[7] for v in _sorted_fallback(dev, ts, ty, G, slots, P)} == {2}
    ts2, ty2 = synthetic_scores(1 << 20, 0.01, dev, seed=5)
    e2 = _oracle(ts2, ty2)
    slots2, _ = _gathered(dev, ts2, ty2, G)
    assert {v[7] for v in _sorted_fallback(dev, ts2, ty2, G, slots2, e2["P"] + 1)} == {2}
    assert {v[7] for v in _sorted_fallback(dev, ts2, ty2, G, slots2, e2["P"])} == {1}
    ts3, ty3 = synthetic_scores(400_000, 0.55, dev, seed=99)
    e3 = _oracle(ts3, ty3)
    slots3, _ = _gathered(dev, ts3, ty3, G)
    assert {v[7] for v in _sorted_fallback(dev, ts3, ty3, G, slots3, e3["P"])} == {2}


@pytest.mark.parametrize("n,p", [(400_000, 0.55), (1 << 19, 0.45)])
@pytest.mark.timeout(300)
def test_two_step_table_past_index_capacity(dev, n, p):
    """a table larger than the count index can hold while no slot overflows (uniform
    positives, G = 8): the gather must stop at the index's capacity and every part report
    verdict 2; the sorted path (positives or negatives as the table) gives the oracle's integers."""
    from distributedauc_amd.loader import synthetic_scores

    ts, ty = synthetic_scores(n, p, dev, seed=99)
    e = _oracle(ts, ty)
    G = 8
    assert e["P"] > min(n // 2 + 1, 219_838)
    recs = _two_step(dev, ts, ty, G)
    assert {(v[3], v[4], v[7]) for v in recs} == {(e["P"], 0, 2)}, recs
    assert _sorted_parts(dev, ts, ty, G) == (e["wins"], e["ties"])


def test_two_step_rejects_overlapping_buffers(dev):
    """a record inside the evaluation workspace or the gathered slots is refused
    (DAUC_EINVAL) instead of being zeroed or overwritten mid-evaluation (step 2 and the sorted slot
    fallback alike; the fallback also refuses P < 1)."""
    from distributedauc_amd import _lib, ops

    n, G = 100_003, 2
    g = torch.Generator(device=dev).manual_seed(3)
    ts = torch.rand(n, generator=g, device=dev)
    ty = torch.where(torch.rand(n, generator=g, device=dev) < 0.05, 1, -1).to(torch.int8)
    nb = ops.auc_slot_bytes(n, G)
    slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
    for r in range(G):
        ops.auc_eval_compact_part(ts, ty, r, G, slots[r * nb:(r + 1) * nb])
    L = _lib.load()
    st = torch.cuda.current_stream(dev).cuda_stream
    ws = ops.workspaces.get(dev, "auc_eval", L.dauc_auc_eval_workspace_size(n), st)
    with pytest.raises(_lib.DaucError):
        ops.auc_eval_query_part(ts, ty, 0, G, slots, out=ws[1024:1088].view(torch.int64))
    with pytest.raises(_lib.DaucError):
        ops.auc_eval_query_part(ts, ty, 0, G, slots, out=slots[256:320].view(torch.int64))
    with pytest.raises(_lib.DaucError):
        ops.auc_eval_enqueue(ts, ty, 0, G, out=ws[2048:2112].view(torch.int64))
    # the sorted slot fallback: the same rules, and a table of at least one positive
    with pytest.raises(_lib.DaucError):
        ops.auc_eval_query_part_sorted(ts, ty, 0, G, slots, 100, out=ws[1024:1088].view(torch.int64))
    with pytest.raises(_lib.DaucError):
        ops.auc_eval_query_part_sorted(ts, ty, 0, G, slots, 100, out=slots[256:320].view(torch.int64))
    with pytest.raises(_lib.DaucError):
        ops.auc_eval_query_part_sorted(ts, ty, 0, G, slots, 0)
    # the slots are untouched by the refused calls: the evaluation still gives the oracle's counts
    e = _oracle(ts, ty)
    recs = [_query(dev, ts, ty, r, G, slots) for r in range(G)]
    assert (sum(v[0] for v in recs), sum(v[1] for v in recs)) == (e["wins"], e["ties"])


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_worker(rank, world, port, q):
    import traceback

    import torch.distributed as dist

    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from distributedauc_amd.auc import ExactAUC
        from distributedauc_amd.loader import synthetic_scores

        ts, ty = synthetic_scores(1 << 24, 0.01, dev)
        e = _oracle(ts, ty)
        ev = ExactAUC(world=world, rank=rank)  # SHARD_MIN = 2^24: sharded
        c = ev.counts(ty, ts)
        assert ev.last_mode == "sharded"
        assert (c["wins"], c["ties"], c["P"], c["N"]) == (e["wins"], e["ties"], e["P"], e["N"]), (c, e)
        # labels that differ in rank 1's own slice (queried by rank 0): both ranks raise
        y3 = ty.clone()
        if rank == 1:
            y3[(1 << 23) + 12345:(1 << 23) + 12345 + 64] = 1
        with pytest.raises(RuntimeError, match="disagree"):
            ev.counts(y3, ts)
        # different lengths: equal slot sizes, the collectives complete, both ranks raise (shard_min
        # 0: both lengths take the sharded path -- lengths on either side of SHARD_MIN would not)
        m = (1 << 24) - (0 if rank == 0 else 4096)
        with pytest.raises(RuntimeError, match="different lengths"):
            ExactAUC(world=world, rank=rank, shard_min=0).counts(ty[:m], ts[:m])
        assert ev.counts(ty, ts) == c  # the group is still usable
        # tie-heavy scores (bf16-rounded): verdict 2, then the sorted two-step fallback over the
        # gathered slots (the distinct-key index) on both ranks
        tb = ts.bfloat16().float()
        eb = _oracle(tb, ty)
        cb = ev.counts(ty, tb)
        assert (cb["wins"], cb["ties"], cb["P"], cb["N"]) == (eb["wins"], eb["ties"], eb["P"], eb["N"]), (cb, eb)
        dist.destroy_process_group()
        q.put((rank, None))
    except BaseException:
        q.put((rank, traceback.format_exc()))


@pytest.mark.timeout(400)
def test_exact_auc_sharded_two_gloo_ranks_2e24():
    """ExactAUC's sharded path (compaction of its slice, the slot all-gather, the query of the
    next slice, the record all-gather) as 2 real processes on cuda:0 over gloo, at configs[3]'s
    2^24 scores: the oracle's counts on both ranks; mismatching inputs raise on both."""
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(360)
    res = []
    while not q.empty():
        res.append(q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = [e for _, e in res if e]
    assert not errs, "\n".join(errs)
    assert sorted(r for r, _ in res) == list(range(world))


@pytest.mark.parametrize("mults", [(5, 6, 8), (9, 12, 14), (15,)])
def test_two_step_slotted_cells_of_many_keys(dev, mults):
    """The slotted build (round 6): a cell's keys 0-3 in its primary window, 4-7 in its secondary
    window, 8-14 in its tertiary run; a cell of 15+ keys refuses the index (verdict 2, as the direct
    build's nibble did). Positives repeating one score value `m` times put m keys in one cell; the
    negatives include that value (ties) and its neighbours. Bit-exact against the C oracle for G = 2,
    3 (verdict 1 below 15 keys; verdict 2, then the sorted path, at 15)."""
    from distributedauc_amd import ops

    rng = np.random.default_rng(77 + sum(mults))
    n = 400_003
    # random scores below 0.25, the repeated values at 0.3 / 0.4 / 0.5: their top buckets hold
    # nothing else, so each value's cell holds exactly its m keys
    s = (rng.random(n, dtype=np.float32) * np.float32(0.25)).astype(np.float32)
    y = np.where(rng.random(n) < 0.05, 1, -1).astype(np.int8)
    pos = np.flatnonzero(y == 1)
    neg = np.flatnonzero(y == -1)
    at = 0
    for j, m in enumerate(mults):
        v = np.float32(0.3 + 0.1 * j)
        s[pos[at:at + m]] = v
        at += m
        s[neg[100 * j:100 * j + 7]] = v                                     # ties
        s[neg[100 * j + 7:100 * j + 9]] = np.nextafter(v, np.float32(1))     # just above
        s[neg[100 * j + 9:100 * j + 11]] = np.nextafter(v, np.float32(0))    # just below
    ts, ty = torch.from_numpy(s).to(dev), torch.from_numpy(y).to(dev)
    e = _oracle(ts, ty)
    for G in (2, 3):
        recs = _two_step(dev, ts, ty, G)
        verdicts = {v[7] for v in recs}
        if max(mults) >= 15:
            assert verdicts == {2}, recs
            assert _sorted_parts(dev, ts, ty, G) == (e["wins"], e["ties"])
        else:
            assert verdicts == {1}, recs
            assert (sum(v[0] for v in recs), sum(v[1] for v in recs)) == (e["wins"], e["ties"]), (G, recs)


def test_two_step_second_query_without_step1(dev):
    """Step 2 consumes the build state step 1 prepared in the workspace: a second
    dauc_auc_eval_query_part without a new dauc_auc_eval_compact_part must not count the keys twice --
    it reports verdict 2, and the blocking sorted path gives the exact integers."""
    from distributedauc_amd import ops

    n, G = 300_007, 2
    g = torch.Generator(device=dev).manual_seed(9)
    ts = torch.rand(n, generator=g, device=dev)
    ty = torch.where(torch.rand(n, generator=g, device=dev) < 0.02, 1, -1).to(torch.int8)
    e = _oracle(ts, ty)
    nb = ops.auc_slot_bytes(n, G)
    slots = torch.empty(nb * G, dtype=torch.uint8, device=dev)
    for r in range(G):
        ops.auc_eval_compact_part(ts, ty, r, G, slots[r * nb:(r + 1) * nb])
    first = ops.auc_eval_query_part(ts, ty, G - 1, G, slots).cpu().tolist()
    again = ops.auc_eval_query_part(ts, ty, G - 1, G, slots).cpu().tolist()
    assert first[7] == 1 and again[7] == 2, (first, again)
    assert again[3] == first[3] == e["P"] and again[4] == 0
    assert _sorted_parts(dev, ts, ty, G) == (e["wins"], e["ties"])
    # a fresh step 1 re-arms it
    recs = _two_step(dev, ts, ty, G)
    assert {v[7] for v in recs} == {1}
    assert (sum(v[0] for v in recs), sum(v[1] for v in recs)) == (e["wins"], e["ties"])
