"""Oracle parity at every BASELINE.json config's full workload, on the reference's
own triples where the snapshot has them (tests/golden/<dataset>_ids.npz), plus the upstream loss
flags (model.py:4-44 / upstream KGEModel.train_step: adversarial vs mean, temperature, uni_weight,
L3 regularisation) against the oracle's fp64 autograd.

Full-size kernels run over the whole [B, N] batch; the fp64 oracle checks sampled rows (the
oracle's [rows, N, d] gather finishes in seconds), and every row in chunks for C2 (scores and row outputs, both
modes) and C3 / C4 (scores, one mode each). Bar: |got - ref| <= 1e-4 max(1, |ref|)."""
import os
import types

import numpy as np
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd import evaluate, ops
from customknowledgegraphembedding_amd._lib import FN_IDS
from customknowledgegraphembedding_amd.distributed import HipShardKernels, shard_bounds
from oracle import kge_oracle as O
from tests.conftest import rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4
GOLD = os.path.join(os.path.dirname(__file__), "golden")
ROWS = [0, 1, 97, 256, 510, 511]


def _triples(key):
    with np.load(os.path.join(GOLD, f"{key}_ids.npz")) as z:
        return z["triples"].astype(np.int64)


def _batch(key, E, B, N, seed):
    tri = _triples(key)
    perm = np.random.RandomState(0).permutation(len(tri))
    pos = torch.from_numpy(tri[perm[seed * B:(seed + 1) * B]])
    neg = torch.from_numpy(np.random.RandomState(2 + seed).randint(E, size=(B, N)))
    return pos, neg


def _step_forward_vs_oracle(name, E, R, d, gamma, de, dr, tr, key, B, N):
    m = kge.TFKGEModel(name, E, R, d, gamma, double_entity_embedding=de, double_relation_embedding=dr,
                       triple_relation_embedding=tr, device=DEV, seed=0)
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    pos, neg = _batch(key, E, B, N, seed=1)
    fn = FN_IDS[name]
    for mode in (0, 1):
        out_neg, out_pos, ns, ps = ops.step_forward_raw(fn, mode, m.entity_embedding.detach(),
                                                        m.relation_embedding.detach(), m._rel_off, pos.to(DEV),
                                                        neg.to(DEV), m._D, m._gamma_f, m._range_f)
        torch.cuda.synchronize()
        ref_s = O.score(name, ent, rel, pos[ROWS], neg[ROWS], mode, gamma, m._range_f).numpy()
        assert rel_close(ns.cpu().numpy()[ROWS], ref_s) <= TOL, (name, mode)
        ref_n = O.tf_call(name, ent, rel, pos[ROWS], neg[ROWS], mode, gamma, m._range_f).numpy()[:, 0]
        ref_p = O.tf_call(name, ent, rel, pos[ROWS], neg[ROWS], 3, gamma, m._range_f).numpy()[:, 0]
        assert rel_close(out_neg.cpu().numpy()[ROWS], ref_n) <= TOL, (name, mode)
        assert rel_close(out_pos.cpu().numpy()[ROWS], ref_p) <= TOL, (name, mode)
    return m, pos, neg


def test_c2_wn18rr_interht_full_size_real_positives():
    """C2: WN18RR InterHT d=1000 -de -tr gamma=24, B=512, N=256, positives from train.txt."""
    _step_forward_vs_oracle("InterHT", 40943, 11, 1000, 24.0, True, False, True, "wn18rr", 512, 256)


def _all_rows_vs_oracle(name, E, R, d, gamma, de, dr, tr, key, B, N, modes, outputs, chunk=64, useful=False):
    """Every batch row of a full-size step (not the sampled ROWS) against the fp64 oracle, in chunks of rows
    so the oracle's [chunk, N, d] gathers stay small: the raw scores, and with `outputs` the two calls' row
    outputs (self-adversarial negative term, positive log-sigmoid). `useful`: the row outputs from the selected
    branch only (O.adv_reduce of the reference scores, O.score in mode 3: tf_call's values whenever no branch
    is NaN, at a third of the oracle's work)."""
    m = kge.TFKGEModel(name, E, R, d, gamma, double_entity_embedding=de, double_relation_embedding=dr,
                       triple_relation_embedding=tr, device=DEV, seed=0)
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    pos, neg = _batch(key, E, B, N, seed=3)
    fn = FN_IDS[name]
    for mode in modes:
        out_neg, out_pos, ns, _ = ops.step_forward_raw(fn, mode, m.entity_embedding.detach(),
                                                       m.relation_embedding.detach(), m._rel_off, pos.to(DEV),
                                                       neg.to(DEV), m._D, m._gamma_f, m._range_f)
        torch.cuda.synchronize()
        ns, out_neg, out_pos = ns.cpu().numpy(), out_neg.cpu().numpy(), out_pos.cpu().numpy()
        worst = 0.0
        for r0 in range(0, B, chunk):
            rows = slice(r0, min(B, r0 + chunk))
            ref_s = O.score(name, ent, rel, pos[rows], neg[rows], mode, gamma, m._range_f).numpy()
            worst = max(worst, rel_close(ns[rows], ref_s))
            if outputs and useful:
                ref_n = O.adv_reduce(torch.from_numpy(ref_s)).numpy()[:, 0]
                ref_p = torch.nn.functional.logsigmoid(
                    O.score(name, ent, rel, pos[rows], neg[rows], 3, gamma, m._range_f)).numpy()[:, 0]
                worst = max(worst, rel_close(out_neg[rows], ref_n), rel_close(out_pos[rows], ref_p))
            elif outputs:
                ref_n = O.tf_call(name, ent, rel, pos[rows], neg[rows], mode, gamma, m._range_f).numpy()[:, 0]
                ref_p = O.tf_call(name, ent, rel, pos[rows], neg[rows], 3, gamma, m._range_f).numpy()[:, 0]
                worst = max(worst, rel_close(out_neg[rows], ref_n), rel_close(out_pos[rows], ref_p))
        assert worst <= TOL, (name, mode, worst)


def test_c2_every_row_full_size():
    """C2 (the headline): all 512 rows x 256 negatives of a full-size WN18RR InterHT step, both modes, scores
    and both calls' row outputs against the fp64 oracle (the tile order's whole output, not sampled rows)."""
    _all_rows_vs_oracle("InterHT", 40943, 11, 1000, 24.0, True, False, True, "wn18rr", 512, 256, (0, 1), True)


def test_c3_every_row_full_size():
    """C3: every row of a full-size FB15k-237 RotatE step, both modes, raw scores and both calls' row outputs
    against the fp64 oracle."""
    _all_rows_vs_oracle("RotatE", 14541, 237, 1000, 9.0, True, False, False, "fb15k237", 512, 256, (0, 1), True,
                        useful=True)


def test_c4_every_row_full_size():
    """C4 (unsharded): every row of a full-size YAGO3-10 DistMult N = 1 024 step, both modes, raw scores and both
    calls' row outputs against the fp64 oracle."""
    _all_rows_vs_oracle("DistMult", 123182, 37, 500, 24.0, False, False, False, "yago3_10", 512, 1024, (0, 1), True,
                        chunk=32, useful=True)


def test_c2_xcd_phases_bitwise():
    """The XCD-sliced step swept in phases (the C2 table exceeds the Infinity Cache: 4 phases by default)
    scores every candidate with the same code: outputs bitwise equal for 1, 2, 3, 4 and 8 phases, and equal
    to the plain scorer's scores."""
    name, E, R, d = "InterHT", 40943, 11, 1000
    m = kge.TFKGEModel(name, E, R, d, 24.0, double_entity_embedding=True, triple_relation_embedding=True,
                       device=DEV, seed=0)
    pos, neg = _batch("wn18rr", E, 512, 256, seed=2)
    pos, neg = pos.to(DEV), neg.to(DEV)
    ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
    fn = FN_IDS[name]
    for mode in (0, 1):
        outs = []
        for ph in (1, 2, 3, 4, 8):  # the phases belong to the XCD-sliced form (the default is the tile form)
            outs.append(ops.step_forward_raw(fn, mode, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f,
                                             forms=dict(step_order="xcd", xcd_phases=ph))[:3])
        want_s = ops.score_indexed_raw(fn, mode, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f)
        torch.cuda.synchronize()
        for o in outs:
            assert all(torch.equal(x, y) for x, y in zip(o, outs[0])), mode
        assert torch.equal(outs[0][2], want_s), mode


def test_c3_fb15k237_rotate_full_size():
    """C3: FB15k-237 RotatE d=1000 -de, E=14541, R=237, B=512, N=256 (valid+test positives)."""
    _step_forward_vs_oracle("RotatE", 14541, 237, 1000, 9.0, True, False, False, "fb15k237", 512, 256)


def test_c4_yago3_10_distmult_full_size_unsharded_and_sharded8():
    """C4: YAGO3-10 DistMult d=500, E=123182, N=1024, B=512: the unsharded step forward against the
    oracle, and the row-sharded owner-computes kernels at a simulated world of 8 (shard_bounds over
    8 ranks, one device): the 8 partial score blocks sum to the unsharded scores bitwise."""
    E, R, d, B, N = 123182, 37, 500, 512, 1024
    m, pos, neg = _step_forward_vs_oracle("DistMult", E, R, d, 24.0, False, False, False, "yago3_10", B, N)
    fn = FN_IDS["DistMult"]
    ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
    posd, negd = pos.to(DEV), neg.to(DEV)
    for mode in (0, 1):
        want = ops.score_indexed_raw(fn, mode, ent, rel, 0, posd, negd, d, m._gamma_f, m._range_f)
        qcol = 2 if mode == 0 else 0
        qe = torch.zeros(B, d, device=DEV)
        total = torch.zeros_like(want)
        for r in range(8):
            lo, hi = shard_bounds(E, 8, r)
            part = torch.zeros(B, d, device=DEV)
            HipShardKernels.gather_rows(ent[lo:hi].contiguous(), lo, posd[:, qcol:], 3, B, part)
            qe += part
        for r in range(8):
            lo, hi = shard_bounds(E, 8, r)
            out = torch.empty_like(want)
            HipShardKernels.score_sharded(fn, mode, qe, rel, 0, ent[lo:hi].contiguous(), lo, posd, negd, d,
                                          m._gamma_f, m._range_f, 0.0, out)
            total += out
        assert torch.equal(total, want), mode


def test_c5_fb15k_filtered_ranks_full_entity_set():
    """C5: FB15k all-entity eval, DistMult d=1000 (SURVEY §8 assumption), 14951 entities: filtered
    ranks of sampled valid.txt queries (filter = valid.txt, the split the snapshot holds) against the
    oracle's argsort restatement of upstream test_step, exactly."""
    E, R, d = 14951, 1345, 1000
    m = kge.KGEModel("DistMult", E, R, d, 24.0, device=DEV, seed=0)
    true = _triples("fb15k")
    q = true[np.random.RandomState(5).choice(len(true), 6, replace=False)]
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    for mode in ("head-batch", "tail-batch"):
        ptr, ids = evaluate.build_filter(q, mode, true)
        pos = torch.from_numpy(q).to(DEV)
        S = evaluate.score_all(m, pos, mode)
        col = 0 if mode == "head-batch" else 2
        got = evaluate.rank_filtered(S, pos[:, col].contiguous(), torch.from_numpy(ptr).to(DEV),
                                     torch.from_numpy(ids).to(DEV)).cpu()
        want = O.eval_ranks("DistMult", ent, rel, torch.from_numpy(q), mode, true, 24.0, m._range_f)
        assert torch.equal(got, want), (mode, got, want)


@pytest.mark.parametrize("name", ["DistMult", "ComplEx"])
def test_c5_fb15k_filtered_ranks_512_queries(name):
    """C5 at the bench's query scale: 512 valid.txt queries per mode through test_step's own path (entity planes
    made once, query planes, the bf16x3 plane GEMM, kge_rank_filtered) against O.eval_ranks_dense (S = Q . E^T
    in fp64; pinned to the per-query eval_ranks in test_oracle.py). Every rank must lie in the oracle's [lo, hi]
    under the GEMM's accuracy bound (1e-6 sum|q e| per score: the GEMM's accuracy), and equal the oracle's rank
    exactly wherever no candidate's fp64 margin to the truth is within the two scores' measured errors |S - S64|
    (there the fp32 comparisons are the fp64 ones, so this checks the counting and the filter); at least 95 % of the
    queries must be decided that way."""
    E, R, d = 14951, 1345, 1000
    de = name == "ComplEx"
    m = kge.KGEModel(name, E, R, d, 24.0, double_entity_embedding=de, double_relation_embedding=de, device=DEV,
                     seed=0)
    true = _triples("fb15k")
    q = true[np.random.RandomState(7).choice(len(true), 512, replace=False)]
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    planes = evaluate.entity_planes(m)
    assert planes is not None
    for mode in ("head-batch", "tail-batch"):
        ptr, ids = evaluate.build_filter(q, mode, true)
        pos = torch.from_numpy(q).to(DEV)
        S = evaluate.score_all(m, pos, mode, planes=planes)
        col = 0 if mode == "head-batch" else 2
        got = evaluate.rank_filtered(S, pos[:, col].contiguous(), torch.from_numpy(ptr).to(DEV),
                                     torch.from_numpy(ids).to(DEV)).cpu()
        qt = torch.from_numpy(q)
        want, lo, hi = O.eval_ranks_dense(name, ent, rel, qt, mode, true)
        assert bool(((lo <= got) & (got <= hi)).all()), (name, mode)
        err = (S.detach().cpu().double() - O.eval_scores_dense(name, ent, rel, qt, mode)).abs()
        want2, lo2, hi2 = O.eval_ranks_dense(name, ent, rel, qt, mode, true, atol=err + 1e-30)
        decided = lo2 == hi2
        assert torch.equal(want2, want)
        assert bool(((lo2 <= got) & (got <= hi2)).all()), (name, mode)
        assert torch.equal(got[decided], want[decided]), (name, mode)
        assert float(decided.double().mean()) >= 0.95, (name, mode, int(decided.sum()))
        assert int(want.max()) > 100  # the ranks span the table, not only the top


# ------------------------------------------------------------------------------------------------
# upstream loss flags (model.py:4-44; upstream KGEModel.train_step) vs the oracle's fp64 autograd
# ------------------------------------------------------------------------------------------------
class _NoStep:
    """An optimizer that keeps the gradients for inspection (zero_grad, then a no-op step)."""

    def __init__(self, params):
        self.params = list(params)

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def step(self):
        pass


@pytest.mark.parametrize("name", ["RotatE", "TransE", "DistMult", "ComplEx"])
@pytest.mark.parametrize("adv,temp,uni,reg", [(False, 1.0, False, 0.0), (True, 0.5, False, 0.0),
                                              (True, 1.0, True, 0.0), (True, 1.0, False, 1e-3),
                                              (False, 1.0, True, 2e-3), (True, 2.0, True, 1e-3)])
@pytest.mark.parametrize("mode", ["head-batch", "tail-batch"])
def test_upstream_train_step_flags_loss_and_grads(name, adv, temp, uni, reg, mode):
    de = name in ("RotatE", "ComplEx")
    dr = name == "ComplEx"
    E, R, d, B, N, gamma = 120, 6, 24, 10, 17, 9.0
    m = kge.KGEModel(name, E, R, d, gamma, double_entity_embedding=de, double_relation_embedding=dr, device=DEV,
                     seed=4)
    ent = m.entity_embedding.detach().cpu().double().requires_grad_(True)
    rel = m.relation_embedding.detach().cpu().double().requires_grad_(True)
    g = np.random.RandomState(9)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(g.randint(E, size=(B, N)))
    w = torch.from_numpy(g.uniform(0.1, 1.0, size=(B,))).float()
    args = types.SimpleNamespace(negative_adversarial_sampling=adv, adversarial_temperature=temp, uni_weight=uni,
                                 regularization=reg)

    def it():
        while True:
            yield pos, neg, w, mode

    opt = _NoStep(m.parameters())
    log = kge.KGEModel.train_step(m, opt, it(), args)
    ref = O.upstream_train_loss(name, ent, rel, pos, neg, w.double(), mode, gamma, m._range_f,
                                adversarial=adv, temperature=temp, uni_weight=uni, regularization=reg)
    ref.backward()
    assert log["loss"] == pytest.approx(ref.item(), rel=1e-5, abs=1e-6)
    for got, want in ((m.entity_embedding.grad, ent.grad), (m.relation_embedding.grad, rel.grad)):
        scale = float(want.abs().max().clamp_min(1e-12))
        assert float((got.cpu().double() - want).abs().max()) <= 1e-4 * scale, (name, adv, temp, uni, reg)
