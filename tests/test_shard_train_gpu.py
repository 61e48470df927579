"""GPU tests of the row-sharded train step (kge_shard_train_*; distributed.ShardedKGE.train_step):
W ranks simulated as threads of one process on one device (ThreadComm), each holding a block of
entity rows. The step must equal supervisor.py:15-26 run by W replicas on their own batches with
SUM gradient aggregation and Keras Adam (tf.distribute apply_gradients), computed by the oracle in
fp64 autograd: sum over replicas of O.tf_train_loss -> gradients -> O.keras_adam_step."""
import numpy as np
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd.distributed import ShardedKGE, ThreadComm, run_threads, shard_bounds
from customknowledgegraphembedding_amd.optim import Adam
from customknowledgegraphembedding_amd.supervisor import Strategy, Sum, Trainer
from oracle import kge_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = {"InterHT": (True, False, True), "TransE": (False, False, False), "DistMult": (False, False, False),
       "ComplEx": (True, True, False), "RotatE": (True, False, False)}


def _batches(E, R, Bg, N, steps, seed):
    g = np.random.RandomState(seed)
    out = []
    for i in range(steps):
        pos = torch.from_numpy(np.stack([g.randint(E, size=Bg), g.randint(R, size=Bg), g.randint(E, size=Bg)], 1))
        neg = torch.from_numpy(g.randint(E, size=(Bg, N)))
        w = torch.from_numpy(g.uniform(0.1, 1.0, size=(Bg,))).float()
        out.append((pos, neg, w, i % 2))
    return out


def _sharded_run(name, E, R, d, gamma, W, batches, lr, seed=7, **opts):
    de, dr, tr = CFG[name]
    comm = ThreadComm(W)
    ranks = [ShardedKGE(name, E, R, d, gamma, de, dr, tr, device=DEV, seed=seed, world=W, rank=r, comm=comm)
             for r in range(W)]
    for sk in ranks:
        sk.configure_optimizer(lr=lr)
        for k, v in opts.items():
            setattr(sk, k, v)
    dev_batches = [(p.to(DEV), n.to(DEV), w.to(DEV), m) for p, n, w, m in batches]
    losses = []
    for pos, neg, w, mode in dev_batches:
        out = run_threads([lambda sk=sk: sk.train_step(pos, neg, w, mode) for sk in ranks])
        torch.cuda.synchronize()
        losses.append([float(x) for x in out])
    ent = torch.cat([sk.shard.cpu() for sk in ranks])
    rels = [sk.relation_embedding.cpu() for sk in ranks]
    return losses, ent, rels, ranks


def _oracle_run(name, E, R, d, gamma, W, batches, lr, seed=7, loss_fn=None):
    de, dr, tr = CFG[name]
    ref = kge.TFKGEModel(name, E, R, d, gamma, de, dr, tr, device="cpu", seed=seed)
    ent = ref.entity_embedding.detach().double()
    rel = ref.relation_embedding.detach().double()
    st = {}
    losses = []
    for t, (pos, neg, w, mode) in enumerate(batches, start=1):
        e = ent.clone().requires_grad_(True)
        r = rel.clone().requires_grad_(True)
        Bh = pos.shape[0] // W
        per = []
        for h in range(W):
            sl = slice(h * Bh, (h + 1) * Bh)
            if loss_fn is None:
                lh = O.tf_train_loss(name, e, r, pos[sl], neg[sl], w[sl].double(), torch.tensor([mode] * Bh), gamma,
                                     ref._range_f)
            else:
                lh = loss_fn(e, r, pos[sl], neg[sl], w[sl].double(), mode, ref._range_f)
            per.append(lh)
        total = sum(per)
        total.backward()
        losses.append([x.item() for x in per])
        for key, p, gr in (("e", ent, e.grad), ("r", rel, r.grad)):
            mm, vv = st.get(key, (torch.zeros_like(p), torch.zeros_like(p)))
            p2, mm, vv = O.keras_adam_step(p, gr, mm, vv, t, lr)
            st[key] = (mm, vv)
            if key == "e":
                ent = p2.detach()
            else:
                rel = p2.detach()
    return losses, ent, rel


@pytest.mark.parametrize("name", list(CFG))
@pytest.mark.parametrize("W", [1, 2, 4])
def test_sharded_train_step_matches_replicated_sum_oracle(name, W):
    E, R, d, Bh, N, gamma, lr = 97, 5, 40, 6, 24, 9.0, 2e-3
    batches = _batches(E, R, W * Bh, N, 3, seed=W)
    la, ent, rels, _ = _sharded_run(name, E, R, d, gamma, W, batches, lr)
    lb, ent_ref, rel_ref = _oracle_run(name, E, R, d, gamma, W, batches, lr)
    # every rank returns its own replica's loss
    np.testing.assert_allclose(np.array(la), np.array(lb), rtol=1e-4, atol=1e-6)
    for r in rels[1:]:
        assert torch.equal(r, rels[0])  # the replicated relation table stays identical on every rank
    assert float((ent.double() - ent_ref).abs().max()) <= 5e-2 * lr, name
    assert float((rels[0].double() - rel_ref).abs().max()) <= 5e-2 * lr, name


@pytest.mark.parametrize("adv,detach", [(True, True), (False, False)])
def test_sharded_train_step_upstream_reductions(adv, detach):
    """Detached self-adversarial weights (upstream) and the mean reduction."""
    name, E, R, d, Bh, N, gamma, lr, W = "RotatE", 83, 4, 32, 5, 20, 9.0, 2e-3, 2
    batches = _batches(E, R, W * Bh, N, 2, seed=11)
    la, ent, rels, _ = _sharded_run(name, E, R, d, gamma, W, batches, lr, adversarial=adv, detach=detach)

    def loss_fn(e, r, pos, neg, w, mode, rng):
        return O.upstream_train_loss(name, e, r, pos, neg, w, mode, gamma, rng, adversarial=adv)

    lb, ent_ref, rel_ref = _oracle_run(name, E, R, d, gamma, W, batches, lr, loss_fn=loss_fn)
    np.testing.assert_allclose(np.array(la), np.array(lb), rtol=1e-4, atol=1e-6)
    assert float((ent.double() - ent_ref).abs().max()) <= 5e-2 * lr
    assert float((rels[0].double() - rel_ref).abs().max()) <= 5e-2 * lr


def test_sharded_world1_equals_single_gpu_train_step():
    """At one rank the sharded step is kge_train_step's algebra: same losses to fp32 rounding and
    tables within a small multiple of lr of Trainer's fused single-GPU step."""
    name, E, R, d, B, N, gamma, lr = "InterHT", 120, 5, 64, 16, 40, 9.0, 2e-3
    batches = _batches(E, R, B, N, 3, seed=3)
    la, ent, rels, _ = _sharded_run(name, E, R, d, gamma, 1, batches, lr)
    m = kge.TFKGEModel(name, E, R, d, gamma, True, False, True, device=DEV, seed=7)
    tr = Trainer(Strategy(), None, m, Adam(m.parameters(), lr=lr), Sum())
    data = iter([(p, n, w.reshape(-1, 1), torch.tensor([md] * B)) for p, n, w, md in batches])
    lb = [float(tr.train_step(data)) for _ in range(3)]
    np.testing.assert_allclose([x[0] for x in la], lb, rtol=2e-6, atol=1e-7)
    assert float((ent.to(DEV) - m.entity_embedding.detach()).abs().max()) <= 2e-2 * lr
    assert float((rels[0].to(DEV) - m.relation_embedding.detach()).abs().max()) <= 2e-2 * lr


def test_sharded_train_step_deterministic_and_hot_rows():
    """Bitwise reproducible run to run; a tiny table (hot rows: > 64 events per row) at 4 ranks."""
    name, E, R, d, Bh, N, gamma, lr, W = "DistMult", 23, 3, 16, 8, 50, 9.0, 2e-3, 4
    batches = _batches(E, R, W * Bh, N, 2, seed=5)
    a = _sharded_run(name, E, R, d, gamma, W, batches, lr)
    b = _sharded_run(name, E, R, d, gamma, W, batches, lr)
    assert a[0] == b[0]
    assert torch.equal(a[1], b[1])
    lb, ent_ref, rel_ref = _oracle_run(name, E, R, d, gamma, W, batches, lr)
    np.testing.assert_allclose(np.array(a[0]), np.array(lb), rtol=1e-4, atol=1e-6)
    assert float((a[1].double() - ent_ref).abs().max()) <= 5e-2 * lr


def test_sharded_c4_full_size_step_runs_and_matches_sampled_oracle_loss():
    """C4 (YAGO3-10 DistMult d=500, E=123182, N=1024) at a simulated 8-way split, Bg = 8 x 64:
    one step runs, every replica's loss matches the oracle's forward on that replica's batch."""
    E, R, d, N, W, Bh, gamma = 123182, 37, 500, 1024, 8, 64, 24.0
    batches = _batches(E, R, W * Bh, N, 1, seed=2)
    la, _, _, ranks = _sharded_run("DistMult", E, R, d, gamma, W, batches, 1e-4, seed=0)
    ref = kge.TFKGEModel("DistMult", E, R, d, gamma, device="cpu", seed=0)
    ent, rel = ref.entity_embedding.detach().double(), ref.relation_embedding.detach().double()
    pos, neg, w, mode = batches[0]
    for h in (0, 5):
        sl = slice(h * Bh, (h + 1) * Bh)
        want = O.tf_train_loss("DistMult", ent, rel, pos[sl], neg[sl], w[sl].double(), torch.tensor([mode] * Bh),
                               gamma, ref._range_f).item()
        assert la[0][h] == pytest.approx(want, rel=1e-4)
    assert all(sk.shard.shape[0] == shard_bounds(E, W, sk.rank)[1] - shard_bounds(E, W, sk.rank)[0] for sk in ranks)

