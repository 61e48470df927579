"""GPU tests of the row-sharded forward's O(information) exchange (kge_shard_plan,
kge_shard_gather_queries, kge_shard_score, kge_shard_finish; distributed.ShardedKGE.step_forward):
W ranks simulated as threads of one process on one device (ThreadComm: the same all-to-all calls
TorchComm makes over RCCL). Every score has one owner and moves once, so each home rank's scores
must equal the unsharded kernel's bitwise, and its reductions kge_step_forward's."""
import numpy as np
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd import ops
from customknowledgegraphembedding_amd._lib import FN_IDS
from customknowledgegraphembedding_amd.distributed import ShardedKGE, ThreadComm, run_threads
from tests.shard_oracle_backend import OracleShardKernels

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = {"TransE": (False, False, False), "DistMult": (False, False, False), "ComplEx": (True, True, False),
       "RotatE": (True, False, False), "pRotatE": (False, False, False), "InterHT": (True, False, True)}


def _model(name, E, R, d, seed=3):
    de, dr, tr = CFG[name]
    return kge.TFKGEModel(name, E, R, d, 9.0, double_entity_embedding=de, double_relation_embedding=dr,
                          triple_relation_embedding=tr, device=DEV, seed=seed)


def _batch(E, R, Bg, N, seed, bad=False):
    g = np.random.RandomState(seed)
    pos = torch.from_numpy(np.stack([g.randint(E, size=Bg), g.randint(R, size=Bg), g.randint(E, size=Bg)], 1))
    neg = torch.from_numpy(g.randint(E, size=(Bg, N)))
    if bad:  # ids without an owner (TF-GPU gathers a zero row; the sharded path scores them 0)
        neg[1, 0] = E + 5
        neg[Bg - 1, N - 1] = -3
    return pos.to(DEV), neg.to(DEV)


def _ranks(m, W, comm=None):
    mod = float(m.modulus.detach().reshape(-1)[0]) if m.model_name == "pRotatE" else 0.0
    tables = (m.entity_embedding.detach(), m.relation_embedding.detach(), m._gamma_f, m._range_f, mod)
    comm = comm or ThreadComm(W)
    return [ShardedKGE(m.model_name, m.nentity, m.nrelation, m.hidden_dim, m._gamma_f, device=DEV, world=W,
                       rank=r, comm=comm, full_tables=tables) for r in range(W)]


@pytest.mark.parametrize("W,K", [(1, 1), (2, 1), (2, 2), (3, 3), (8, 4), (8, 2)])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("flags", [0, 1])
@pytest.mark.parametrize("N", [70, 300])
def test_plan_matches_restatement(W, K, mode, flags, N):
    """kge_shard_plan's counts, prefixes, query owners / slots and summary equal the CPU restatement (the
    forward's one query column with the head-batch positive on the head's owner, and the train step's two),
    and so does the forward plan's bucket of the first and the last rank (owned candidates grouped by XCD
    slice; the order inside a slice is the LDS atomics' and not specified)."""
    E, R, Bh = 301, 7, 5
    m = _model("DistMult", E, R, 8)
    pos, neg = _batch(E, R, W * Bh, N, seed=W + 10 * K, bad=True)
    ranks = _ranks(m, W)
    for sk in {0: ranks[0], W - 1: ranks[-1]}.values():
        got = sk.kernels.plan(sk, pos, neg, mode, K, flags)
        want = OracleShardKernels.plan(sk, pos.cpu(), neg.cpu(), mode, K, flags)
        for a in ("cnt", "hpre", "qown", "qslot"):
            assert torch.equal(getattr(got, a).cpu().long(), getattr(want, a).long()), a
        gt, gq = got.summary()
        wt, wq = want.summary()
        assert np.array_equal(gt, wt) and np.array_equal(gq, wq)
        if flags:
            assert got.bucket is None
            continue
        start = got.bucket_start.cpu()
        assert torch.equal(start, want.bucket_start), sk.rank
        gb = got.bucket.cpu()
        for g in range(W * Bh):  # a slice's entries in any order (each carries its rank)
            for x in range(8):
                lo, hi = int(start[g, x]), int(start[g, x + 1])
                key = lambda e: sorted(map(tuple, e.tolist()))  # noqa: E731
                assert key(gb[g, lo:hi]) == key(want.bucket[g, lo:hi]), (sk.rank, g, x)


def _check_world(name, W, K, E, R, d, Bh, N, seed, bad=False):
    m = _model(name, E, R, d)
    fn = FN_IDS[name]
    ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
    mod = float(m.modulus.detach().reshape(-1)[0]) if name == "pRotatE" else 0.0
    pos, neg = _batch(E, R, W * Bh, N, seed, bad)
    ranks = _ranks(m, W)
    for mode in (0, 1):
        outs = run_threads([lambda sk=sk: sk.step_forward(pos, neg, mode, chunks=K) for sk in ranks])
        torch.cuda.synchronize()
        want_s = ops.score_indexed_raw(fn, mode, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f, mod)
        want_neg, want_pos, _, _ = ops.step_forward_raw(fn, mode, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f,
                                                        m._range_f, mod)
        valid = (neg >= 0) & (neg < E)
        for r, (o_neg, o_pos, s) in enumerate(outs):
            sl = slice(r * Bh, (r + 1) * Bh)
            assert torch.equal(s, torch.where(valid[sl], want_s[sl], torch.zeros_like(s))), (mode, r)
            assert torch.equal(o_pos, want_pos[sl]), (mode, r)
            if not bad:
                assert torch.equal(o_neg, want_neg[sl]), (mode, r)


@pytest.mark.parametrize("name", list(CFG))
@pytest.mark.parametrize("W,K", [(1, 1), (2, 2), (4, 2)])
def test_sharded_forward_bitwise_every_function(name, W, K):
    """N < 128 (a slice's run well under one 64-lane run)."""
    _check_world(name, W, K, E=997, R=6, d=40, Bh=6, N=37, seed=1)


@pytest.mark.parametrize("name", ["InterHT", "DistMult", "RotatE"])
@pytest.mark.parametrize("W,K", [(2, 1), (4, 4), (8, 4)])
def test_sharded_forward_bitwise_xcd_order(name, W, K):
    """N >= 128: the unsharded reference is the XCD-sliced kernel (compact ranks carried through the
    bucket scorer's per-run row sort)."""
    _check_world(name, W, K, E=5003, R=5, d=64, Bh=8, N=300, seed=2)


def test_sharded_forward_ids_without_owner():
    """Out-of-range candidates score 0 and are never sent; every other score stays bitwise."""
    _check_world("TransE", 4, 2, E=211, R=3, d=16, Bh=4, N=150, seed=4, bad=True)


def test_sharded_forward_plan_made_ahead_and_reused():
    """A plan made one step ahead (the bench's pipelining), also on a side stream, gives the same results
    as an inline one."""
    E, R, d, W, Bh, N = 3001, 5, 32, 4, 8, 200
    m = _model("DistMult", E, R, d)
    pos, neg = _batch(E, R, W * Bh, N, seed=5)
    ranks = _ranks(m, W)
    plans = [sk.plan(pos, neg, 1) for sk in ranks]
    a = run_threads([lambda sk=sk, p=p: sk.step_forward(pos, neg, 1, plan=p) for sk, p in zip(ranks, plans)])
    b = run_threads([lambda sk=sk: sk.step_forward(pos, neg, 1) for sk in ranks])
    side = torch.cuda.Stream()  # plans made on a side stream, waited for by the step's stream
    plans = [sk.plan(pos, neg, 1, stream=side) for sk in ranks]
    c = run_threads([lambda sk=sk, p=p: sk.step_forward(pos, neg, 1, plan=p) for sk, p in zip(ranks, plans)])
    for x, y, z in zip(a, b, c):
        for u, v, t in zip(x, y, z):
            assert torch.equal(u, v) and torch.equal(u, t)


def test_collective_bytes_are_payload_only():
    """Per rank the score all-to-all carries exactly the rank's home scores owned elsewhere, and the query
    all-to-all exactly the other owners' query rows, no padding: O(B) and O(W B) per rank, not O(W B N)."""
    E, R, d, W, Bh, N = 4001, 5, 16, 8, 16, 256
    m = _model("DistMult", E, R, d)
    pos, neg = _batch(E, R, W * Bh, N, seed=6)
    sk = _ranks(m, W)[3]
    plan = sk.plan(pos, neg, 0)
    cb = sk.collective_bytes(plan)
    home = slice(3 * Bh, 4 * Bh)
    cand = torch.cat([neg[home], pos[home, 0:1]], 1)  # head-batch: the positive belongs to its head's owner
    foreign = int(((cand < sk.lo) | (cand >= sk.hi)).sum())
    assert cb["scores"] == foreign * 4
    # the zero-padded reduce-scatter moved W * Bh * (N + 1) floats per rank per step
    assert cb["scores"] < Bh * (N + 1) * 4 < W * Bh * (N + 1) * 4
    # query rows: exactly the batch's tails owned by the other ranks, one row each
    tails = pos[:, 2]
    assert cb["query_rows"] == int(((tails < sk.lo) | (tails >= sk.hi)).sum()) * m.entity_embedding.shape[1] * 4


def test_c4_full_size_simulated_8_ranks():
    """C4 at full size (YAGO3-10 DistMult d=500, E=123182, N=1024, 8 x 512 rows, YAGO positives) through
    the whole 8-rank step on one GPU: every home's scores equal the unsharded kernel's bitwise."""
    with np.load("tests/golden/yago3_10_ids.npz") as z:
        tri = z["triples"].astype(np.int64)
    E, R, d, W, Bh, N = 123182, 37, 500, 8, 512, 1024
    m = kge.TFKGEModel("DistMult", E, R, d, 24.0, device=DEV, seed=0)
    perm = np.random.RandomState(0).permutation(len(tri))[:W * Bh]
    pos = torch.from_numpy(tri[perm]).to(DEV)
    neg = torch.from_numpy(np.random.RandomState(200).randint(E, size=(W * Bh, N))).to(DEV)
    ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
    ranks = _ranks(m, W)
    for mode in (0, 1):
        outs = run_threads([lambda sk=sk: sk.step_forward(pos, neg, mode) for sk in ranks])
        torch.cuda.synchronize()
        want_s = ops.score_indexed_raw(1, mode, ent, rel, 0, pos, neg, d, m._gamma_f, m._range_f)
        want_neg, want_pos, _, _ = ops.step_forward_raw(1, mode, ent, rel, 0, pos, neg, d, m._gamma_f, m._range_f)
        for r, (o_neg, o_pos, s) in enumerate(outs):
            sl = slice(r * Bh, (r + 1) * Bh)
            assert torch.equal(s, want_s[sl]) and torch.equal(o_neg, want_neg[sl]) and torch.equal(o_pos, want_pos[sl])
