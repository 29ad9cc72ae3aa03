"""DDP / FSDP / pipeline / pipeline x DDP engines on CPU (gloo, multi-process) must produce
the same parameters as the single-process engine on the same global batch."""
import itertools
import os

import pytest
import torch

from dist_helpers import run_workers
from dist_workers import (reference_state, worker_ddp, worker_fsdp, worker_fsdp_mem, worker_pipe, worker_scaled)

from distributed_pytorch_cookbook_amd.parallel.pipeline import partition, schedule_1f1b

pytestmark = pytest.mark.slow


def assert_close_sd(a, b, atol=2e-5):
    assert list(a.keys()) == list(b.keys())
    for k in a:
        assert torch.allclose(a[k].float(), b[k].float(), atol=atol, rtol=1e-4), \
            (k, (a[k] - b[k]).abs().max().item())


@pytest.fixture(scope="module")
def ref():
    return reference_state(steps=2)


@pytest.mark.parametrize("reduce_dtype", ["float32"])
def test_ddp_matches_single(tmp_path, ref, reduce_dtype):
    out = tmp_path / "ddp.pt"
    run_workers(worker_ddp, 2, str(out), 2, 0.05, reduce_dtype)
    assert_close_sd(torch.load(out, weights_only=True), ref[0])


# --reduce_dtype bf16 (SURVEY.md §5.8 rule 3) on every gradient collective: the DDP bucket
# all-reduce, the FSDP reduce-scatter and the PP x DP replica all-reduce.  bf16 rounds each
# gradient to 8 significant bits before the sum, so the result is close to, not equal to, the
# f32 single-process one; the engines must also actually reduce in bf16 (checked by the
# deviation being non-zero somewhere for FSDP, whose shards see only reduced gradients)
@pytest.mark.parametrize("kind", ["ddp", "fsdp", "pipe_ddp"])
def test_bf16_gradient_reduction_close_to_f32(tmp_path, ref, kind):
    out = tmp_path / f"{kind}_bf16.pt"
    if kind == "ddp":
        run_workers(worker_ddp, 2, str(out), 2, 0.05, "bfloat16")
        sd = torch.load(out, weights_only=True)
    elif kind == "fsdp":
        run_workers(worker_fsdp, 2, str(out), 2, 1, True, "bfloat16")
        sd = torch.load(out, weights_only=True)
    else:
        run_workers(worker_pipe, 4, str(out), 2, 2, 2, 2, "1f1b", "bfloat16")
        sd = torch.load(out, weights_only=True)["sd"]
    # AdamW normalises each gradient element, so an element whose summed gradient is near zero
    # can flip sign under bf16 rounding and move by up to 2 x lr; the bulk must stay close
    assert list(sd) == list(ref[0])
    diff = torch.cat([(sd[k].float() - ref[0][k].float()).abs().flatten() for k in sd])
    assert diff.max().item() <= 2.5 * 1e-2, diff.max().item()
    assert diff.mean().item() < 1e-3, diff.mean().item()
    assert (diff > 1e-3).float().mean().item() < 0.02
    assert diff.max().item() > 0.0, "bf16 reduction produced the f32 result bit for bit: not reduced in bf16"


@pytest.mark.parametrize("prefetch,reshard", [(1, True), (2, False)])
def test_fsdp_matches_single(tmp_path, ref, prefetch, reshard):
    out = tmp_path / "fsdp.pt"
    run_workers(worker_fsdp, 2, str(out), 2, prefetch, reshard)
    assert_close_sd(torch.load(out, weights_only=True), ref[0])


@pytest.mark.parametrize("schedule,micro", [("1f1b", 4), ("gpipe", 2), ("zb", 4)])
def test_pipeline_matches_single(tmp_path, ref, schedule, micro):
    out = tmp_path / "pp.pt"
    run_workers(worker_pipe, 2, str(out), 2, 2, 1, micro, schedule)
    r = torch.load(out, weights_only=True)
    assert_close_sd(r["sd"], ref[0])


def test_pipeline_three_stages(tmp_path, ref):
    out = tmp_path / "pp3.pt"
    run_workers(worker_pipe, 3, str(out), 2, 3, 1, 4, "1f1b")
    assert_close_sd(torch.load(out, weights_only=True)["sd"], ref[0])


def test_pipe_ddp_mesh_matches_single(tmp_path, ref):
    out = tmp_path / "ppdp.pt"
    run_workers(worker_pipe, 4, str(out), 2, 2, 2, 2, "1f1b")
    assert_close_sd(torch.load(out, weights_only=True)["sd"], ref[0])


@pytest.mark.parametrize("kind", ["ddp", "fsdp", "pipe"])
def test_grad_scaler_engines_match_single(tmp_path, ref, kind):
    out = tmp_path / f"scaled_{kind}.pt"
    run_workers(worker_scaled, 2, str(out), kind)
    assert_close_sd(torch.load(out, weights_only=True), ref[0])


def test_partition_balanced_and_contiguous():
    costs = [0.1] + [1.0] * 24 + [3.5]
    g = partition(costs, 8)
    assert [u for grp in g for u in grp] == list(range(26))
    loads = [sum(costs[u] for u in grp) for grp in g]
    assert max(loads) <= 4.1
    assert g[-1][-1] == 25 and len(g[-1]) < len(g[1])


def test_1f1b_order_counts():
    for st in range(4):
        o = schedule_1f1b(8, st, 4)
        assert [m for k, m in o if k == "F"] == list(range(8))
        assert [m for k, m in o if k == "B"] == list(range(8))
        # at most (stages - stage) micro-batches in flight
        inflight = mx = 0
        for k, _ in o:
            inflight += 1 if k == "F" else -1
            mx = max(mx, inflight)
        assert mx <= 4 - st


def test_comm_bw_bench_runs_on_gloo(tmp_path):
    """bench/comm_bw.py: every collective of the engines, 2 ranks over gloo."""
    import json
    import subprocess
    import sys

    from dist_helpers import ROOT, free_port

    out = tmp_path / "bw.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), f"{ROOT}/bench/comm_bw.py",
           "--cpu", "--sizes_mb", "0.25", "--iters", "2", "--warmup", "1", "--json", str(out)]
    subprocess.run(cmd, check=True, timeout=180, capture_output=True, env={**os.environ, "OMP_NUM_THREADS": "1"})
    rows = json.loads(out.read_text())
    assert {r["op"] for r in rows} == {"all_reduce", "all_gather", "reduce_scatter", "broadcast", "sendrecv"}
    assert all(r["busbw_GBps"] > 0 and r["world"] == 2 for r in rows)


def test_pipe_ddp_default_mesh_is_pp2():
    from distributed_pytorch_cookbook_amd.recipes import pipe_mesh

    assert pipe_mesh("pipe_ddp", 8) == (2, 4)
    assert pipe_mesh("pipe_ddp", 4) == (2, 2)
    assert pipe_mesh("pipe_ddp", 1) == (1, 1)
    assert pipe_mesh("pipe", 8) == (8, 1)
    assert pipe_mesh("pipe_ddp", 8, dp_size=2) == (4, 2)


def test_run_schedule_is_the_tested_schedule():
    """The engine executes exactly schedule_1f1b / schedule_gpipe: record the op order the
    executor calls on a 4-stage pipeline (no communication: a recording P2P)."""
    from distributed_pytorch_cookbook_amd.parallel.pipeline import run_schedule, schedule_1f1b, schedule_gpipe

    class RecP2P:
        def __init__(self):
            self.posts = []

        def post(self, **kw):
            self.posts.append({k: v is not None for k, v in kw.items()})

            class R:
                def get(self_):
                    return torch.zeros(1)
            rp, rn = kw.get("recv_prev_shape"), kw.get("recv_next_shape")
            return (R() if rp is not None else None), (R() if rn is not None else None)

        def drain(self):
            pass

    for sched in (schedule_1f1b, schedule_gpipe):
        for st in range(4):
            order = sched(8, st, 4)
            seen = []
            p2p = RecP2P()
            run_schedule(order, st == 0, st == 3, lambda m, x: seen.append(("F", m)) or torch.zeros(1),
                         lambda m, g: seen.append(("B", m)) or torch.zeros(1), p2p, (1,))
            assert seen == order
            # every send posted exactly once: 8 forward outputs (not the last stage) and 8
            # input gradients (not the first stage)
            n_send = sum(p.get("send_next", False) for p in p2p.posts), sum(p.get("send_prev", False) for p in p2p.posts)
            assert n_send == ((8 if st < 3 else 0), (8 if st > 0 else 0))
            n_recv = (sum(p.get("recv_prev_shape", False) for p in p2p.posts),
                      sum(p.get("recv_next_shape", False) for p in p2p.posts))
            assert n_recv == ((8 if st > 0 else 0), (8 if st < 3 else 0))


def test_fsdp_memory_bounded(tmp_path):
    """FSDP backward keeps at most prefetch + 2 full-unit buffers (weights + gradients) alive:
    a unit's gradient is released as soon as its reduce-scatter is enqueued."""
    out = tmp_path / "fsdp_mem.pt"
    run_workers(worker_fsdp_mem, 2, str(out))
    r = torch.load(out, weights_only=True)
    for prefetch, peak in r.items():
        assert peak <= prefetch + 2, (prefetch, peak)


@pytest.mark.parametrize("kind", ["ddp", "fsdp", "pipe"])
def test_stream_check_engines_and_unwaited_collective(tmp_path, kind):
    """with the stream-order check on, DDP / FSDP / pipeline steps leave no
    asynchronous collective un-waited, and one that is never waited on is reported."""
    from dist_workers import worker_stream_check

    out = tmp_path / "sc.pt"
    run_workers(worker_stream_check, 2, str(out), kind)
    assert torch.load(out, weights_only=True)["caught"]


def test_fsdp_forced_sharded_path_matches_fast_path():
    """--force_dist_path: the N > 1 FSDP code path (full-unit gathers, unit gradients,
    reduce-scatters, replicated-vector all-reduce) at one rank gives the fast path's result."""
    from dist_workers import LR, full_batch, make_model

    from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine

    res = []
    for forced in (False, True):
        eng = FSDPEngine(make_model(), "cpu", lr=LR, force_sharded=forced)
        assert eng.store.sharded == forced
        for s in range(2):
            eng.train_step(*full_batch(step=s))
        res.append(eng.full_state_dict())
    assert_close_sd(res[0], res[1], atol=1e-6)


@pytest.mark.parametrize("pp,dp,micro,sched", [(2, 1, 4, "zb"), (4, 1, 8, "zb"), (2, 2, 4, "zb"), (4, 1, 8, "zb2")])
def test_zero_bubble_equals_1f1b_exactly(tmp_path, pp, dp, micro, sched):
    """The zero-bubble schedule (B / W split, W passes deferred) reorders work, not arithmetic:
    the weight gradients of a unit are still accumulated micro-batch by micro-batch in order, so
    the trained parameters equal 1F1B's bit for bit (gloo, 2 / 4 stages, and a 2 x 2 mesh whose
    DP buckets launch from the deferred W passes)."""
    a, b = tmp_path / "zb.pt", tmp_path / "1f1b.pt"
    run_workers(worker_pipe, pp * dp, str(a), 2, pp, dp, micro, sched)
    run_workers(worker_pipe, pp * dp, str(b), 2, pp, dp, micro, "1f1b")
    za, zb_ = torch.load(a, weights_only=True)["sd"], torch.load(b, weights_only=True)["sd"]
    assert list(za) == list(zb_)
    for k in za:
        assert torch.equal(za[k], zb_[k]), k


def test_zero_bubble_orders():
    """schedule_zb: every F / B / W of every micro-batch exactly once, B after F, W after B, 1F1B's
    F / B order (mem 2: twice its warm-up) and so at most (mem x) 1F1B's activations in flight;
    deadlock-free under RCCL's blocking p2p as run_schedule issues
    it (p2p_deadlock_free, which 1F1B / GPipe also pass); and a smaller modelled bubble than
    1F1B under the cost model -- at PP = 8, M = 32 within 10 % of the bubble-free time."""
    from distributed_pytorch_cookbook_amd.parallel.pipeline import (bubble_factor, fb_order, p2p_deadlock_free,
                                                                    schedule_gpipe, schedule_zb)

    for p, M, c, mem in itertools.product((2, 3, 4, 8), (1, 2, 3, 8, 16), ((1.0, 1.0, 1.0), (1.0, 1.4, 1.0), (0.5, 2.0, 1.5)),
                                          (1, 2)):
        if True:
            if True:
                orders = [schedule_zb(M, s, p, costs=[c] * p, mem=mem) for s in range(p)]
                for s, o in enumerate(orders):
                    for kind in "FBW":
                        assert [m for k, m in o if k == kind] == list(range(M)), (p, M, s, kind)
                    pos = {op: i for i, op in enumerate(o)}
                    assert all(pos[("F", m)] < pos[("B", m)] < pos[("W", m)] for m in range(M))
                    # 1F1B's activation bound: at most (stages - stage) micro-batches between F and B
                    inflight = mx = 0
                    for k, _ in o:
                        inflight += 1 if k == "F" else (-1 if k == "B" else 0)
                        mx = max(mx, inflight)
                    assert mx <= mem * (p - s), (p, M, s, mx)
                    # the F / B order is 1F1B's (mem 2: with twice the warm-up forwards)
                    want = schedule_1f1b(M, s, p) if mem == 1 else fb_order(M, s, p, 2 * (p - s) - 1)
                    assert [op for op in o if op[0] != "W"] == want, (p, M, s, mem)
                assert p2p_deadlock_free(orders), (p, M, c, mem)
                assert p2p_deadlock_free([schedule_1f1b(M, s, p) for s in range(p)])
                assert p2p_deadlock_free([schedule_gpipe(M, s, p) for s in range(p)])
    # 1F1B with three times the warm-up forwards is NOT deadlock-free under grouped blocking p2p
    assert not p2p_deadlock_free([fb_order(8, s, 4, 3 * (4 - s) - 1) for s in range(4)])
    # the checker does catch a mis-ordered exchange: stage 0 expects B1 before B0
    bad = [[("F", 0), ("F", 1), ("B", 1), ("B", 0)], [("F", 0), ("B", 0), ("F", 1), ("B", 1)]]
    assert not p2p_deadlock_free(bad)
    for p, M in ((8, 32), (2, 8), (8, 16)):
        costs = [(1.0, 1.2, 1.0)] * p
        assert bubble_factor(M, costs, "zb2") <= bubble_factor(M, costs, "zb") < bubble_factor(M, costs, "1f1b")
    assert bubble_factor(32, [(1.0, 1.0, 1.0)] * 8, "zb") < 1.10
    # the measured GPT-2 medium PP=8 stage costs (F, B, W ms, profiles/r6_pp/): zb2 at M = 16
    assert bubble_factor(16, [(4.30, 5.19, 2.96)] * 8, "zb2") < 1.16


def test_run_schedule_executes_zero_bubble_order():
    """run_schedule executes a zb order op for op (W passes through ``wgrad``), posts every send
    once and each receive in the group of the op BEFORE the next communicating op."""
    from distributed_pytorch_cookbook_amd.parallel.pipeline import run_schedule, schedule_zb

    class RecP2P:
        def __init__(self):
            self.posts = []

        def post(self, **kw):
            self.posts.append({k: v is not None for k, v in kw.items()})

            class R:
                def get(self_):
                    return torch.zeros(1)
            rp, rn = kw.get("recv_prev_shape"), kw.get("recv_next_shape")
            return (R() if rp is not None else None), (R() if rn is not None else None)

        def drain(self):
            pass

    for st in range(4):
        order = schedule_zb(8, st, 4)
        seen = []
        p2p = RecP2P()
        run_schedule(order, st == 0, st == 3, lambda m, x: seen.append(("F", m)) or torch.zeros(1),
                     lambda m, g: seen.append(("B", m)) or torch.zeros(1), p2p, (1,),
                     wgrad=lambda m: seen.append(("W", m)))
        assert seen == order
        n_recv = (sum(p.get("recv_prev_shape", False) for p in p2p.posts),
                  sum(p.get("recv_next_shape", False) for p in p2p.posts))
        assert n_recv == ((8 if st > 0 else 0), (8 if st < 3 else 0))
        # W passes are invisible to the communication: the same groups as the order without them
        # (a W never separates a send from the receive the next communicating op consumes)
        p2 = RecP2P()
        run_schedule([op for op in order if op[0] != "W"], st == 0, st == 3, lambda m, x: torch.zeros(1),
                     lambda m, g: torch.zeros(1), p2, (1,))
        assert p2p.posts == p2.posts, st
