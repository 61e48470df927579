"""RCCL on one GPU: every TorchComm method, and the row-sharded steps' whole collective path, run under
torch.distributed's "nccl" backend (RCCL on ROCm) at world size 1, so the first RCCL call of the
distributed path is not the driver's 8-GPU scaling run (distributed.py TorchComm; the reference's
strategy layer: /root/reference/tensorflow_codes/run.py:8-17).

At W = 1 the all-to-alls move one piece (this rank to itself), the all-gather and all-reduce are copies,
but every call goes through RCCL on device tensors with the same arguments the W > 1 path passes:
uneven split lists, zero-size pieces, async work handles. ShardedKGE with `exchange = True` takes the
multi-rank code path (plan, query exchange, compact scoring, score exchange, finish; the train step's
query exchange, stats all-gather and gradient all-reduce) and must give the unsharded results bitwise."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from customknowledgegraphembedding_amd.distributed import ShardedKGE, TorchComm

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def rccl():
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", world_size=1, rank=0,
                            device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield TorchComm()
    dist.destroy_process_group()


def test_torchcomm_methods_under_rccl(rccl):
    c = rccl
    assert c.world == 1 and c.rank == 0
    dev = torch.device("cuda", 0)
    x = torch.arange(37, dtype=torch.float32, device=dev)
    # all_to_all: the full piece, async, then a zero-size piece (a rank that owns nothing of a chunk)
    out = torch.full_like(x, -1.0)
    h = c.all_to_all(out, x, [37], [37], async_op=True)
    h.wait()
    torch.cuda.synchronize()
    assert torch.equal(out, x)
    empty_in = torch.empty(0, dtype=torch.float32, device=dev)
    empty_out = torch.empty(0, dtype=torch.float32, device=dev)
    c.all_to_all(empty_out, empty_in, [0], [0], async_op=True).wait()
    c.all_to_all(empty_out, empty_in, [0], [0]).wait()
    # int32 pieces (the plans' summaries) and a 2-D view
    xi = torch.arange(12, dtype=torch.int32, device=dev).view(3, 4)
    oi = torch.zeros(12, dtype=torch.int32, device=dev)
    c.all_to_all(oi, xi.view(-1), [12], [12]).wait()
    assert torch.equal(oi.view(3, 4), xi)
    # all_gather_into / all_gather_cat
    g = torch.empty((1, 37), dtype=torch.float32, device=dev)
    c.all_gather_into(g, x)
    assert torch.equal(g[0], x)
    assert torch.equal(c.all_gather_cat(x.view(37, 1))[0, :, 0], x)
    c.all_gather_into(g, x, async_op=True).wait()
    # all_reduce_sum_ (sync and async) and broadcast_
    y = x.clone()
    assert c.all_reduce_sum_(y) is y and torch.equal(y, x)
    c.all_reduce_sum_(y, async_op=True).wait()
    assert torch.equal(y, x)
    assert torch.equal(c.broadcast_(y, 0), x)
    torch.cuda.synchronize()


def _batch(E, R, B, N, seed):
    g = np.random.RandomState(seed)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(g.randint(E, size=(B, N)))
    w = torch.from_numpy(g.uniform(0.1, 1.0, size=B)).float()
    return pos.cuda(), neg.cuda(), w.cuda()


@pytest.mark.parametrize("mode", [0, 1])
def test_sharded_step_forward_through_rccl_equals_unsharded(rccl, mode):
    E, R, d, B, N = 1500, 7, 64, 32, 200
    ref = ShardedKGE("DistMult", E, R, d, 24.0, device="cuda", seed=0)          # W = 1: no exchange
    sk = ShardedKGE("DistMult", E, R, d, 24.0, device="cuda", seed=0, comm=rccl)
    sk.exchange = True                                                              # the W > 1 code path
    pos, neg, _ = _batch(E, R, B, N, 3 + mode)
    a = ref.step_forward(pos, neg, mode)
    plan = sk.plan(pos, neg, mode, stream=torch.cuda.Stream())                     # made ahead, side stream
    b = sk.step_forward(pos, neg, mode, plan=plan)
    c = sk.step_forward(pos, neg, mode)
    torch.cuda.synchronize()
    for x, y, z in zip(a, b, c):
        assert torch.equal(x, y) and torch.equal(x, z)


@pytest.mark.parametrize("name", ["DistMult", "InterHT"])
def test_sharded_train_step_through_rccl_equals_world1(rccl, name):
    E, R, d, B, N = 800, 5, 32, 16, 40
    tr = name == "InterHT"
    runs = []
    for exchange in (False, True):
        sk = ShardedKGE(name, E, R, d, 24.0, double_entity_embedding=tr, triple_relation_embedding=tr,
                        device="cuda", seed=1, comm=rccl if exchange else None)
        sk.exchange = exchange
        sk.configure_optimizer(lr=1e-3)
        losses = []
        for i in range(3):
            pos, neg, w = _batch(E, R, B, N, 10 + i)
            losses.append(sk.train_step(pos, neg, w, i % 2).item())
        torch.cuda.synchronize()
        runs.append((losses, sk.shard.cpu(), sk.relation_embedding.cpu()))
    (l0, e0, r0), (l1, e1, r1) = runs
    assert l0 == l1
    assert torch.equal(e0, e1) and torch.equal(r0, r1)
    assert all(np.isfinite(l0))


def test_native_comm_and_executor_through_rccl(rccl):
    """The native communicator (kge_comm_*: its own RCCL communicator, id broadcast through the nccl process
    group) and the native executor over it: ncclAllToAllv self-pieces (including empty ones), the float
    all-reduce, then a chain of row-sharded steps (each planning the next batch) equal the unsharded fused
    forward bitwise."""
    from customknowledgegraphembedding_amd.distributed import NativeComm
    dev = torch.device("cuda", 0)
    nc = NativeComm(device=dev)
    try:
        assert nc.world == 1 and nc.rank == 0
        x = torch.arange(41, dtype=torch.float32, device=dev)
        out = torch.full_like(x, -1.0)
        nc.all_to_all(out, x, [41], [41])
        empty = torch.empty(0, dtype=torch.float32, device=dev)
        nc.all_to_all(empty, empty, [0], [0])
        y = x.clone()
        nc.all_reduce_sum_(y)
        torch.cuda.synchronize()
        assert torch.equal(out, x) and torch.equal(y, x)
        E, R, d, B, N = 1500, 7, 64, 32, 200
        ref = ShardedKGE("DistMult", E, R, d, 24.0, device="cuda", seed=0)
        sk = ShardedKGE("DistMult", E, R, d, 24.0, device="cuda", seed=0).use_native(nc)
        batches = [(*_batch(E, R, B, N, 20 + i)[:2], i % 2) for i in range(4)]
        sk.plan_native(*batches[0])
        sk.plan_native(*batches[1])
        got = [sk.step_forward(p, n, m, nxt=batches[i + 2] if i + 2 < 4 else None)
               for i, (p, n, m) in enumerate(batches)]
        want = [ref.step_forward(p, n, m) for p, n, m in batches]
        torch.cuda.synchronize()
        for a, b in zip(got, want):
            for u, v in zip(a, b):
                assert torch.equal(u, v)
        for ex in sk._native.values():
            ex.close()
    finally:
        nc.close()


def test_bench_rowshard_multi_checks_itself_through_rccl(rccl):
    """bench.py's N > 1 row-sharded section (rowshard_multi) at world 1 through RCCL: the native communicator's
    known-answer check (ncclCommCount, a rank-tagged all-to-all), both executor forms' outputs equal to the
    torch.distributed path's bitwise, the per-rank diagnosis from the executor's timing events, and the report
    the driver's multi-GPU line carries."""
    import argparse

    import bench
    import customknowledgegraphembedding_amd as kge
    from customknowledgegraphembedding_amd import ops
    bench.kge, bench.ops = kge, ops
    a = argparse.Namespace(steps=3, warmup=1)
    rep = bench.rowshard_multi(bench.WORKLOADS["c4s"], a, 1, 0, torch.device("cuda", 0))
    assert rep["native_status"] == "ok" and rep["native_matches_torchcomm"] is True, rep
    assert rep["n_ranks_seen"] == 1 and rep["selected"] == bench.ROWSHARD_DEFAULT
    assert set(rep["variants"]) == {"torchcomm_python", "one_stream_1chunk", "two_stream_2chunk"}
    (r0,) = rep["per_rank"]
    assert all(r0[k] is not None and r0[k] >= 0 for k in bench.ROWSHARD_RANK_KEYS)
    assert 0 < r0["kernel_busy_us"] <= r0["step_us"]
    sp = r0["spans_of_one_step"]
    assert len(sp["score_us"]) == 1 and len(sp["query_a2a_us"]) == 1
