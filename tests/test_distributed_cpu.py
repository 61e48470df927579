"""World-size-2 gloo test of the row-sharded owner-computes scorer (distributed.ShardedKGE) with
the oracle as each rank's local scorer: the sharded forward must equal the unsharded reference
graph (TF call semantics) for every home row."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from customknowledgegraphembedding_amd.distributed import ShardedKGE, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, name, results, chunks=None, B=3, scheme="owner"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.shard_oracle_backend import OracleShardKernels
        from oracle import kge_oracle as O

        E, R, d, N, gamma = 37, 5, 6, 7, 9.0
        de = name in ("ComplEx", "RotatE", "InterHT")
        sk = ShardedKGE(name, E, R, d, gamma, double_entity_embedding=de,
                        double_relation_embedding=(name == "ComplEx"), triple_relation_embedding=(name == "InterHT"),
                        device="cpu", seed=3, kernels=OracleShardKernels())
        g = np.random.RandomState(8)
        WB = world * B
        pos = torch.from_numpy(np.stack([g.randint(E, size=WB), g.randint(R, size=WB), g.randint(E, size=WB)], 1))
        neg = torch.from_numpy(g.randint(E, size=(WB, N)))
        from customknowledgegraphembedding_amd.model import TFKGEModel
        ref = TFKGEModel(name, E, R, d, gamma, de, name == "ComplEx", name == "InterHT", device="cpu", seed=3)
        ent, rel = ref.entity_embedding.detach().double(), ref.relation_embedding.detach().double()
        home = slice(rank * B, (rank + 1) * B)
        errs = []
        for mode in (0, 1):
            if scheme == "gather":
                out_neg, out_pos, scores = sk.step_forward_gather(pos, neg, mode)
            else:
                out_neg, out_pos, scores = sk.step_forward(pos, neg, mode, chunks=chunks)
            want_s = O.score(name, ent, rel, pos[home], neg[home], mode, gamma, ref._range_f, sk.modulus)
            want_neg = O.tf_call(name, ent, rel, pos[home], neg[home], mode, gamma, ref._range_f, sk.modulus)
            want_pos = O.tf_call(name, ent, rel, pos[home], neg[home], 3, gamma, ref._range_f, sk.modulus)
            errs.append(float((scores.double() - want_s).abs().max()))
            errs.append(float((out_neg.double() - want_neg[:, 0]).abs().max()))
            errs.append(float((out_pos.double() - want_pos[:, 0]).abs().max()))
        results[rank] = max(errs)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["DistMult", "InterHT", "RotatE"])
def test_sharded_owner_computes_world2_gloo(name):
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), name, results), nprocs=world, join=True)
    assert len(results) == world
    for r in range(world):
        assert results[r] < 1e-5, (r, results[r])


@pytest.mark.parametrize("chunks,B", [(1, 4), (2, 4), (3, 4), (4, 5)])
def test_sharded_pipelined_chunks_world2_gloo(chunks, B):
    """Chunked pipeline (async all-reduce per chunk, per-chunk reduce-scatter into the home block):
    any chunk count, including one that does not divide B (falls back to a divisor)."""
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), "DistMult", results, chunks, B), nprocs=world, join=True)
    for r in range(world):
        assert results[r] < 1e-5, (r, results[r])


@pytest.mark.parametrize("name", ["TransE", "InterHT"])
def test_sharded_gather_scheme_world2_gloo(name):
    """The all-to-all row-fetch scheme gives the unsharded results on every home row."""
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), name, results, None, 3, "gather"), nprocs=world, join=True)
    for r in range(world):
        assert results[r] < 1e-5, (r, results[r])


def test_shard_bounds_cover_every_row_once():
    for E, W in ((10, 3), (123182, 8), (7, 8)):
        rows = []
        for r in range(W):
            lo, hi = shard_bounds(E, W, r)
            rows.extend(range(lo, hi))
        assert rows == list(range(E))


def _train_worker(rank, world, port, name, results, adv=True, detach=False):
    """World-`world` gloo run of ShardedKGE.train_step (the oracle stand-in as the local kernels):
    three steps on a global batch of world x Bh rows, against the oracle's replicated-SUM step (each
    replica's TF loss on its own batch, summed gradients, Keras Adam) in fp64."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.shard_oracle_backend import OracleShardKernels
        from oracle import kge_oracle as O
        from customknowledgegraphembedding_amd.model import TFKGEModel

        E, R, d, Bh, N, gamma, lr = 29, 4, 6, 3, 7, 9.0, 1e-2
        de, dr, tr = name in ("ComplEx", "RotatE", "InterHT"), name == "ComplEx", name == "InterHT"
        sk = ShardedKGE(name, E, R, d, gamma, de, dr, tr, device="cpu", seed=3, kernels=OracleShardKernels())
        sk.adversarial, sk.detach = adv, detach
        sk.configure_optimizer(lr=lr)
        g = np.random.RandomState(8)
        Bg = world * Bh
        steps = []
        for i in range(3):
            pos = torch.from_numpy(np.stack([g.randint(E, size=Bg), g.randint(R, size=Bg), g.randint(E, size=Bg)], 1))
            neg = torch.from_numpy(g.randint(E, size=(Bg, N)))
            w = torch.from_numpy(g.uniform(0.1, 1.0, size=Bg)).float()
            steps.append((pos, neg, w, i % 2))
        losses = [float(sk.train_step(p, n, w, m)) for p, n, w, m in steps]
        # the oracle: W replicas, SUM of their gradients, Keras Adam
        ref = TFKGEModel(name, E, R, d, gamma, de, dr, tr, device="cpu", seed=3)
        ent, rel = ref.entity_embedding.detach().double(), ref.relation_embedding.detach().double()
        st, ref_losses = {}, []
        for t, (pos, neg, w, mode) in enumerate(steps, start=1):
            e, r = ent.clone().requires_grad_(True), rel.clone().requires_grad_(True)
            per = []
            for h in range(world):
                sl = slice(h * Bh, (h + 1) * Bh)
                if adv and not detach:
                    per.append(O.tf_train_loss(name, e, r, pos[sl], neg[sl], w[sl].double(), [mode], gamma,
                                               ref._range_f))
                else:
                    per.append(O.upstream_train_loss(name, e, r, pos[sl], neg[sl], w[sl].double(), mode, gamma,
                                                     ref._range_f, adversarial=adv))
            sum(per).backward()
            ref_losses.append(per[rank].item())
            for key, p, gr in (("e", ent, e.grad), ("r", rel, r.grad)):
                mm, vv = st.get(key, (torch.zeros_like(p), torch.zeros_like(p)))
                p2, mm, vv = O.keras_adam_step(p, gr, mm, vv, t, lr)
                st[key] = (mm, vv)
                if key == "e":
                    ent = p2.detach()
                else:
                    rel = p2.detach()
        results[rank] = (max(abs(a - b) / max(1.0, abs(b)) for a, b in zip(losses, ref_losses)),
                         float((sk.shard.double() - ent[sk.lo:sk.hi]).abs().max()) / lr,
                         float((sk.relation_embedding.double() - rel).abs().max()) / lr)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("DistMult", 2), ("InterHT", 2), ("RotatE", 3), ("ComplEx", 2)])
def test_sharded_train_step_world_gloo(name, world):
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_train_worker, args=(world, _free_port(), name, results), nprocs=world, join=True)
    for r in range(world):
        lerr, eerr, rerr = results[r]
        assert lerr < 1e-5 and eerr < 1e-3 and rerr < 1e-3, (r, results[r])


@pytest.mark.parametrize("adv,detach", [(True, True), (False, False)])
def test_sharded_train_step_upstream_reductions_gloo(adv, detach):
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_train_worker, args=(2, _free_port(), "TransE", results, adv, detach), nprocs=2, join=True)
    for r in range(2):
        lerr, eerr, rerr = results[r]
        assert lerr < 1e-5 and eerr < 1e-3 and rerr < 1e-3, (r, results[r])


def _trainer_worker(rank, world, port, results):
    """Trainer (supervisor.py:5-58 mirror) at world 2: the fused path row-shards the entity table;
    each rank feeds ITS OWN replica batch; after training the synced model equals the oracle's
    replicated-SUM Keras step on every rank, and the Sum metric is W * sum of the replica losses."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.shard_oracle_backend import OracleShardKernels
        from oracle import kge_oracle as O
        from customknowledgegraphembedding_amd.model import TFKGEModel
        from customknowledgegraphembedding_amd.optim import Adam
        from customknowledgegraphembedding_amd.supervisor import Strategy, Sum, Trainer

        name, E, R, d, B, N, gamma, lr = "InterHT", 31, 3, 6, 3, 5, 9.0, 1e-2
        m = TFKGEModel(name, E, R, d, gamma, True, False, True, device="cpu", seed=5)
        g = np.random.RandomState(4)
        glob = []
        for i in range(2):
            pos = torch.from_numpy(np.stack([g.randint(E, size=world * B), g.randint(R, size=world * B),
                                             g.randint(E, size=world * B)], 1))
            neg = torch.from_numpy(g.randint(E, size=(world * B, N)))
            w = torch.from_numpy(g.uniform(0.1, 1.0, size=(world * B, 1))).float()
            glob.append((pos, neg, w, i % 2))
        mine = [(p[rank * B:(rank + 1) * B], n[rank * B:(rank + 1) * B], w[rank * B:(rank + 1) * B],
                 torch.tensor([md] * B)) for p, n, w, md in glob]
        tr = Trainer(Strategy(), mine, m, Adam(m.parameters(), lr=lr), Sum(), shard_kernels=OracleShardKernels())
        assert tr.sharded is not None
        it = iter(mine)
        for _ in range(2):
            tr.train_step(it)
        tr.sync_model()
        ref = TFKGEModel(name, E, R, d, gamma, True, False, True, device="cpu", seed=5)
        ent, rel = ref.entity_embedding.detach().double(), ref.relation_embedding.detach().double()
        st, total = {}, 0.0
        for t, (pos, neg, w, mode) in enumerate(glob, start=1):
            e, r = ent.clone().requires_grad_(True), rel.clone().requires_grad_(True)
            per = [O.tf_train_loss(name, e, r, pos[h * B:(h + 1) * B], neg[h * B:(h + 1) * B],
                                   w[h * B:(h + 1) * B].double(), [mode], gamma, ref._range_f) for h in range(world)]
            sum(per).backward()
            total += world * sum(x.item() for x in per)
            for key, p, gr in (("e", ent, e.grad), ("r", rel, r.grad)):
                mm, vv = st.get(key, (torch.zeros_like(p), torch.zeros_like(p)))
                p2, mm, vv = O.keras_adam_step(p, gr, mm, vv, t, lr)
                st[key] = (mm, vv)
                if key == "e":
                    ent = p2.detach()
                else:
                    rel = p2.detach()
        results[rank] = (float((m.entity_embedding.detach().double() - ent).abs().max()) / lr,
                         float((m.relation_embedding.detach().double() - rel).abs().max()) / lr,
                         abs(float(tr.metrics.result()) - total) / max(1.0, abs(total)))
    finally:
        dist.destroy_process_group()


def test_trainer_multi_replica_row_sharded_gloo():
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_trainer_worker, args=(2, _free_port(), results), nprocs=2, join=True)
    for r in range(2):
        eerr, rerr, merr = results[r]
        assert eerr < 1e-3 and rerr < 1e-3 and merr < 1e-5, (r, results[r])


@pytest.mark.parametrize("world,chunks", [(4, 2), (3, 3), (4, 1)])
def test_sharded_owner_computes_more_ranks_gloo(world, chunks):
    """World 3 and 4 over gloo: chunks of several whole homes (world 4, 2 chunks), one home per chunk, and
    one chunk for all; the all-gather / all-to-all splits come from the plan, with no padding of scores."""
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), "TransE", results, chunks, 2), nprocs=world, join=True)
    assert len(results) == world
    for r in range(world):
        assert results[r] < 1e-5, (r, results[r])


def test_step_forward_rejects_a_plan_of_another_batch_or_mode():
    """step_forward(plan=...) checks the plan's mode, shape and tensors against the step's (a plan made for
    another step would give wrong scores with no error): ValueError before any collective."""
    from shard_oracle_backend import OracleShardKernels
    E, R, d, Bg, N = 40, 3, 8, 4, 6
    sk = ShardedKGE("DistMult", E, R, d, 24.0, device="cpu", seed=0, world=2, rank=0, comm=object(),
                    kernels=OracleShardKernels())
    g = np.random.RandomState(0)
    pos = torch.from_numpy(np.stack([g.randint(E, size=Bg), g.randint(R, size=Bg), g.randint(E, size=Bg)], 1))
    neg = torch.from_numpy(g.randint(E, size=(Bg, N)))
    plan = sk.plan(pos, neg, 1, chunks=1)
    with pytest.raises(ValueError, match="mode"):
        sk.step_forward(pos, neg, 0, plan=plan)
    with pytest.raises(ValueError, match="other pos/neg"):
        sk.step_forward(pos.clone(), neg.clone(), 1, plan=plan)
    with pytest.raises(ValueError, match="batch"):
        sk.step_forward(pos, neg[:, :N - 1].contiguous(), 1, plan=plan)
