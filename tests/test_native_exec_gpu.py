"""GPU tests of the native row-sharded step (kge_shard_exec_*, csrc/kge_comm.hip; ShardedKGE.use_native):
one C call per rank-step, the plan of the next batch made inside it, the collectives issued from C++.
W ranks run as threads of one process on one device with loopback communicators (device copies ordered
like a real collective), each rank on its own compute stream. Every score has one owner and moves once, so
each home rank's outputs must equal the unsharded kernels' bitwise, as the TorchComm / ThreadComm path's do
(tests/test_shard_exchange_gpu.py). The same executor over RCCL at world 1: tests/test_rccl_gpu.py."""
import numpy as np
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd import ops
from customknowledgegraphembedding_amd._lib import FN_IDS, KGEHipError
from customknowledgegraphembedding_amd.distributed import LoopbackGroup, ShardedKGE, run_threads

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120)]
DEV = "cuda"
CFG = {"DistMult": (False, False, False), "InterHT": (True, False, True), "RotatE": (True, False, False),
       "TransE": (False, False, False), "ComplEx": (True, True, False)}


def _model(name, E, R, d, seed=3):
    de, dr, tr = CFG[name]
    return kge.TFKGEModel(name, E, R, d, 9.0, double_entity_embedding=de, double_relation_embedding=dr,
                          triple_relation_embedding=tr, device=DEV, seed=seed)


def _batch(E, R, Bg, N, seed):
    g = np.random.RandomState(seed)
    pos = torch.from_numpy(np.stack([g.randint(E, size=Bg), g.randint(R, size=Bg), g.randint(E, size=Bg)], 1))
    neg = torch.from_numpy(g.randint(E, size=(Bg, N)))
    return pos.to(DEV), neg.to(DEV)


def _native_ranks(m, W, group, one_stream=False):
    tables = (m.entity_embedding.detach(), m.relation_embedding.detach(), m._gamma_f, m._range_f, 0.0)
    ranks = [ShardedKGE(m.model_name, m.nentity, m.nrelation, m.hidden_dim, m._gamma_f, device=DEV, world=W,
                        rank=r, full_tables=tables) for r in range(W)]
    for r, sk in enumerate(ranks):
        sk.use_native(group.comm(r) if group is not None else None, one_stream=one_stream)
    return ranks


def _want(m, pos, neg, mode):
    fn = FN_IDS[m.model_name]
    ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
    s = ops.score_indexed_raw(fn, mode, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f)
    o_neg, o_pos, _, _ = ops.step_forward_raw(fn, mode, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f)
    return s, o_neg, o_pos


def _run(ranks, batches, K=None, ahead=2):
    """Every rank steps through `batches` ([(pos, neg, mode)]) on its own stream: the first `ahead` batches
    planned up front, then each step planning the batch `ahead` steps later (the plan-ahead chain); returns
    per batch the ranks' outputs."""
    W = len(ranks)
    streams = [torch.cuda.Stream() for _ in range(W)]
    torch.cuda.synchronize()

    def go(r):
        outs = []
        with torch.cuda.stream(streams[r]):
            for b in batches[:ahead]:
                ranks[r].plan_native(*b, chunks=K)
            for i, (pos, neg, mode) in enumerate(batches):
                nxt = batches[i + ahead] if ahead and i + ahead < len(batches) else None
                outs.append(ranks[r].step_forward(pos, neg, mode, chunks=K, nxt=nxt))
        return outs

    res = run_threads([lambda r=r: go(r) for r in range(W)])
    torch.cuda.synchronize()
    return [[res[r][i] for r in range(W)] for i in range(len(batches))]


def _check(m, ranks, batches, K=None, ahead=2):
    W = len(ranks)
    Bh = batches[0][0].shape[0] // W
    for (pos, neg, mode), outs in zip(batches, _run(ranks, batches, K, ahead)):
        s, o_neg, o_pos = _want(m, pos, neg, mode)
        for r, (g_neg, g_pos, g_s) in enumerate(outs):
            sl = slice(r * Bh, (r + 1) * Bh)
            assert torch.equal(g_s, s[sl]), (mode, r)
            assert torch.equal(g_pos, o_pos[sl]), (mode, r)
            assert torch.equal(g_neg, o_neg[sl]), (mode, r)


@pytest.mark.parametrize("name", ["DistMult", "InterHT", "RotatE"])
def test_world1_device_copies_bitwise(name):
    """W = 1 without a communicator (the pieces are device copies): five batches, planned inline or chained
    through the plan-ahead one to three batches ahead, both modes, equal the unsharded fused forward bitwise."""
    E, R, d, Bg, N = 3001, 5, 48, 24, 300
    m = _model(name, E, R, d)
    ranks = _native_ranks(m, 1, None)
    batches = [(*_batch(E, R, Bg, N, seed=s), s % 2) for s in range(5)]
    for ahead in (0, 1, 2, 3):  # planned inline, one, two and three batches ahead
        _check(m, ranks, batches, ahead=ahead)


@pytest.mark.parametrize("W,K,one", [(2, 1, False), (2, 2, False), (4, 2, False), (8, 2, False), (8, 4, False),
                                     (4, 2, True), (8, 1, True)])
@pytest.mark.parametrize("name", ["DistMult", "InterHT"])
def test_loopback_ranks_bitwise(name, W, K, one):
    """W loopback ranks (one thread and one stream each): every home's outputs equal the unsharded kernels'
    bitwise, over a chain of batches alternating head / tail (each step plans the next one); with the
    collectives on a communication stream or on the step's own (KGE_EXEC_ONE_STREAM)."""
    E, R, d, Bh, N = 5003, 5, 64, 8, 300
    m = _model(name, E, R, d)
    group = LoopbackGroup(W)
    try:
        ranks = _native_ranks(m, W, group, one_stream=one)
        batches = [(*_batch(E, R, W * Bh, N, seed=10 + s), s % 2) for s in range(4)]
        _check(m, ranks, batches, K)
        for sk in ranks:
            for ex in sk._native.values():
                ex.close()
    finally:
        group.close()


@pytest.mark.parametrize("name", ["TransE", "ComplEx"])
def test_loopback_small_n_every_layout(name):
    """N < 128 and the other split layouts: 3 ranks, one chunk per home."""
    E, R, d, Bh, N = 997, 6, 40, 6, 37
    m = _model(name, E, R, d)
    group = LoopbackGroup(3)
    try:
        ranks = _native_ranks(m, 3, group)
        _check(m, ranks, [(*_batch(E, R, 3 * Bh, N, seed=1), 0), (*_batch(E, R, 3 * Bh, N, seed=2), 1)], 3)
        for sk in ranks:
            for ex in sk._native.values():
                ex.close()
    finally:
        group.close()


def test_c4_full_size_8_loopback_ranks():
    """C4 at full size (YAGO3-10 DistMult d=500, E=123182, N=1024, 8 x 512 rows, YAGO positives) through the
    native executor's 8-rank step: every home's outputs equal the unsharded kernels' bitwise."""
    with np.load("tests/golden/yago3_10_ids.npz") as z:
        tri = z["triples"].astype(np.int64)
    E, R, d, W, Bh, N = 123182, 37, 500, 8, 512, 1024
    m = kge.TFKGEModel("DistMult", E, R, d, 24.0, device=DEV, seed=0)
    perm = np.random.RandomState(0).permutation(len(tri))[:2 * W * Bh]
    negs = np.random.RandomState(200).randint(E, size=(2 * W * Bh, N))
    batches = [(torch.from_numpy(tri[perm[i * W * Bh:(i + 1) * W * Bh]]).to(DEV),
                torch.from_numpy(negs[i * W * Bh:(i + 1) * W * Bh]).to(DEV), i) for i in range(2)]
    group = LoopbackGroup(W)
    try:
        ranks = _native_ranks(m, W, group)
        _check(m, ranks, batches)
        for sk in ranks:
            for ex in sk._native.values():
                ex.close()
    finally:
        group.close()


def test_step_of_another_batch_than_the_planned_one_is_rejected():
    E, R, d, Bg, N = 1001, 3, 16, 8, 130
    m = _model("DistMult", E, R, d)
    sk = _native_ranks(m, 1, None)[0]
    a, b = _batch(E, R, Bg, N, seed=1), _batch(E, R, Bg, N, seed=2)
    sk.step_forward(a[0], a[1], 0, nxt=(a[0], a[1], 1))  # plans batch a, tail-batch, for the next step
    sk.plan_native(b[0], b[1], 0)
    sk.plan_native(b[0], b[1], 1)  # three plans wait: a step with another next batch has no slot for it
    with pytest.raises(KGEHipError, match="every plan slot"):
        sk.plan_native(a[0], a[1], 0)
    with pytest.raises(KGEHipError, match="another batch or mode"):
        sk.step_forward(b[0], b[1], 1)
    with pytest.raises(KGEHipError, match="another batch or mode"):
        sk.step_forward(a[0], a[1], 0)
    sk.step_forward(a[0], a[1], 1)  # the planned batches, in order
    sk.step_forward(b[0], b[1], 0)
    sk.step_forward(b[0], b[1], 1)
    torch.cuda.synchronize()
