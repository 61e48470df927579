"""Parity at TRAINED-range inputs (the other parity tests draw tables at their initialisation range).

Training leaves the embeddings unconstrained, so the kernels that moved onto the hardware transcendentals
(RotatE's relation phases and pRotatE's per-element sin on v_sin_f32 / v_cos_f32 after one v_fract_f32 on the
revolutions; the row reductions' exp / log on v_exp_f32 / v_log_f32) are checked here where those inputs are
large: RotatE phases up to +-8 pi, +-160 pi (80 revolutions) and +-1 200 pi (past the instruction's +-256
revolutions, which the fract keeps it inside); pRotatE arguments of ~12 pi and ~500 rad; row reductions and the
fused train step on scores spread over +-200. Reference: the fp64 oracle (oracle/kge_oracle.py, restating
upstream RotatE / pRotatE and model.py:168-171's self-adversarial reduction) on the same fp32 inputs.
Bar: |got - ref| <= 1e-4 max(1, |ref|) for scores and row outputs (the north star's), and a RELATIVE 1e-4 for
the log-sigmoid of well-separated rows (tiny values, which an absolute bar would not see)."""
import numpy as np
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd import ops
from customknowledgegraphembedding_amd._lib import FN_IDS
from customknowledgegraphembedding_amd.optim import Adam
from oracle import kge_oracle as O
from tests.conftest import rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4


def _case(name, E, R, d, gamma, B, N, seed, ent_scale=1.0, rel_scale=1.0):
    em, rm = {"RotatE": (2, 1), "pRotatE": (1, 1), "DistMult": (1, 1), "ComplEx": (2, 2)}[name]
    ent, rel, rng = O.make_tables(E, R, em * d, rm * d, gamma, d, seed=seed)
    g = np.random.RandomState(seed)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(g.randint(E, size=(B, N)))
    return (ent * ent_scale).float(), (rel * rel_scale).float(), pos, neg, rng


def _indexed_vs_oracle(name, ent, rel, pos, neg, d, gamma, rng, mod=0.0):
    worst = 0.0
    for mode in (0, 1, 3):
        ref = O.score(name, ent.double(), rel.double(), pos, neg, mode, gamma, rng, mod).numpy()
        got = ops.score_indexed_raw(FN_IDS[name], mode, ent.to(DEV), rel.to(DEV), 0, pos.to(DEV), neg.to(DEV), d,
                                    gamma, rng, mod).cpu().numpy()
        worst = max(worst, rel_close(got, ref))
    return worst


def _step_vs_oracle(name, ent, rel, pos, neg, d, gamma, rng, mod=0.0):
    """kge_step_forward (at N >= 128 the tile kernel + the row reductions): raw scores and both calls' row
    outputs against the oracle's TF-semantics call."""
    worst = 0.0
    for mode in (0, 1):
        out_neg, out_pos, ns, _ = ops.step_forward_raw(FN_IDS[name], mode, ent.to(DEV), rel.to(DEV), 0, pos.to(DEV),
                                                       neg.to(DEV), d, gamma, rng, mod)
        torch.cuda.synchronize()
        e, r = ent.double(), rel.double()
        ref_s = O.score(name, e, r, pos, neg, mode, gamma, rng, mod).numpy()
        ref_n = O.tf_call(name, e, r, pos, neg, mode, gamma, rng, mod).numpy()[:, 0]
        ref_p = O.tf_call(name, e, r, pos, neg, 3, gamma, rng, mod).numpy()[:, 0]
        worst = max(worst, rel_close(ns.cpu().numpy(), ref_s), rel_close(out_neg.cpu().numpy(), ref_n),
                    rel_close(out_pos.cpu().numpy(), ref_p))
    return worst


@pytest.mark.parametrize("turns", [4, 80, 600])
def test_trained_range_rotate_phases(turns):
    """RotatE with the relation table scaled so the phases r / (range / pi) reach +-2 pi `turns` (4: +-8 pi;
    80: the ADVICE's ~500 rad; 600: past v_sin_f32's +-256 revolutions)."""
    name, d, gamma = "RotatE", 1000, 9.0
    ent, rel, pos, neg, rng = _case(name, 500, 7, d, gamma, 24, 160, seed=turns, rel_scale=2.0 * turns)
    ph = rel.double().abs().max().item() / (rng / np.pi)
    assert ph > 1.8 * np.pi * turns  # the phases do reach the range under test
    assert _indexed_vs_oracle(name, ent, rel, pos, neg, d, gamma, rng) <= TOL
    assert _step_vs_oracle(name, ent, rel, pos, neg, d, gamma, rng) <= TOL


@pytest.mark.parametrize("scale", [4.0, 160.0])
def test_trained_range_protate_arguments(scale):
    """pRotatE with both tables scaled so |z| = |phase(h) +- phase(r) - phase(t)| reaches ~12 pi (scale 4) and
    ~500 rad (scale 160)."""
    name, d, gamma = "pRotatE", 1000, 9.0
    ent, rel, pos, neg, rng = _case(name, 500, 7, d, gamma, 24, 160, seed=int(scale), ent_scale=scale,
                                    rel_scale=scale)
    mod = 0.5 * rng
    zmax = 3 * ent.double().abs().max().item() / (rng / 3.14159262)
    assert zmax > 2.5 * np.pi * scale
    assert _indexed_vs_oracle(name, ent, rel, pos, neg, d, gamma, rng, mod) <= TOL
    assert _step_vs_oracle(name, ent, rel, pos, neg, d, gamma, rng, mod) <= TOL


def _spread_scale(name, ent, rel, pos, neg, d, gamma, rng, target=100.0):
    """The common factor on both tables that gives the scores a standard deviation of ~target
    (DistMult / ComplEx scores are cubic in it)."""
    s = O.score(name, ent.double(), rel.double(), pos[:8], neg[:8], 1, gamma, rng).numpy()
    return float((target / s.std()) ** (1.0 / 3.0))


@pytest.mark.parametrize("name", ["DistMult", "ComplEx"])
@pytest.mark.parametrize("N", [256, 1024])
def test_trained_range_step_reductions(name, N):
    """The step's row reductions (neg_rows_kernel after the tile kernel: softmax(s) . logsigmoid(-s) on
    v_exp_f32 / v_log_f32) and the positives' log-sigmoid on scores spread over ~+-200."""
    d, gamma = 250, 24.0
    ent, rel, pos, neg, rng = _case(name, 2000, 9, d, gamma, 32, N, seed=N)
    k = _spread_scale(name, ent, rel, pos, neg, d, gamma, rng)
    ent, rel = ent * k, rel * k
    s = O.score(name, ent.double(), rel.double(), pos, neg, 1, gamma, rng).numpy()
    assert s.max() > 150 and s.min() < -150
    assert _step_vs_oracle(name, ent, rel, pos, neg, d, gamma, rng) <= TOL


def test_reductions_wide_scores_and_small_row_losses():
    """kge_neg_reduce (adversarial and mean) on scores over +-200 against fp64; and rows whose every score is
    far below 0 (a well-separated negative row: logsigmoid(-s) ~ -e^s, 1e-9 .. 1e-18) to 1e-4 RELATIVE."""
    g = np.random.RandomState(5)
    s = torch.from_numpy(g.uniform(-200, 200, size=(64, 300))).float()
    for adv in (True, False):
        got = ops.neg_reduce_raw(s.to(DEV), 1.0, adv).cpu().numpy()
        ref = (O.adv_reduce(s.double()) if adv else O.mean_reduce(s.double())).numpy().reshape(-1)
        assert rel_close(got, ref) <= TOL, adv
    small = torch.from_numpy(g.uniform(-40.0, -20.0, size=(16, 256))).float()
    for adv in (True, False):
        got = ops.neg_reduce_raw(small.to(DEV), 1.0, adv).cpu().double().numpy()
        ref = (O.adv_reduce(small.double()) if adv else O.mean_reduce(small.double())).numpy().reshape(-1)
        assert np.all(ref < 0) and np.all(np.abs(ref) < 1e-8)
        assert float(np.max(np.abs(got - ref) / np.abs(ref))) <= TOL, adv


@pytest.mark.parametrize("name", ["DistMult", "ComplEx"])
def test_trained_range_fused_train_step(name):
    """kge_train_step (the fused forward's online-softmax gradient weights on the hardware exp / log / rcp) on
    scores spread over ~+-200: loss within 1e-4 of the oracle's fp64 TF-semantics loss, and one Keras Adam step
    of both tables within 5e-2 lr of the oracle's."""
    d, gamma, lr, E, R, B, N = 250, 24.0, 1e-3, 600, 5, 16, 200
    m = kge.TFKGEModel(name, E, R, d, gamma, double_entity_embedding=name == "ComplEx",
                       double_relation_embedding=name == "ComplEx", device=DEV, seed=3)
    g = np.random.RandomState(8)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(g.randint(E, size=(B, N)))
    w = torch.from_numpy(g.uniform(0.2, 1.0, size=(B, 1))).float()
    ent0 = m.entity_embedding.detach().cpu().double()
    rel0 = m.relation_embedding.detach().cpu().double()
    k = _spread_scale(name, ent0.float(), rel0.float(), pos, neg, d, gamma, m._range_f)
    with torch.no_grad():
        m.entity_embedding.mul_(k)
        m.relation_embedding.mul_(k)
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    s = O.score(name, ent, rel, pos, neg, 1, gamma, m._range_f).numpy()
    assert s.max() > 150 and s.min() < -150
    opt = Adam(m.parameters(), lr=lr)
    loss = float(m.train_step_fused(pos.to(DEV), neg.to(DEV), w.to(DEV), 1, opt))
    e = ent.clone().requires_grad_(True)
    r = rel.clone().requires_grad_(True)
    ref = O.tf_train_loss(name, e, r, pos, neg, w.double(), torch.tensor([1] * B), gamma, m._range_f)
    ref.backward()
    assert abs(loss - ref.item()) <= TOL * max(1.0, abs(ref.item())), (loss, ref.item())
    for p_got, p0, gr in ((m.entity_embedding, ent, e.grad), (m.relation_embedding, rel, r.grad)):
        p1, _, _ = O.keras_adam_step(p0, gr, torch.zeros_like(p0), torch.zeros_like(p0), 1, lr)
        assert (p_got.detach().cpu().double() - p1).abs().max().item() <= 5e-2 * lr


@pytest.mark.parametrize("mode", [0, 1])
def test_fused_train_step_well_separated_rows(mode):
    """the fused train forward's gradient weights on rows whose every score is far below 0 (e^s < 2^-24:
    logsigmoid(-s) ~ -e^s, which log(1 + e) flushed to 0, dropping the T f term of the weight and the T R_b term of
    the row's gradient). Keras Adam's epsilon is set to the median |gradient| of the oracle's step, so the update
    lr g / (|g| + eps) follows the gradient's magnitude (not only its sign) where |g| ~ eps: a factor-2 error there
    moves a parameter by ~0.15 lr. One step of both tables within 5e-2 lr of the oracle's."""
    name, E, R, d, B, N, lr = "TransE", 300, 5, 64, 24, 160, 1e-3
    m = kge.TFKGEModel(name, E, R, d, 0.0, device=DEV, seed=7)
    g = np.random.RandomState(11)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(g.randint(E, size=(B, N)))
    w = torch.from_numpy(g.uniform(0.2, 1.0, size=(B, 1))).float()
    ent0 = m.entity_embedding.detach().cpu().double()
    rel0 = m.relation_embedding.detach().cpu().double()
    s0 = O.score(name, ent0, rel0, pos, neg, mode, 0.0)
    k = 17.5 / float(-s0.max())  # every score at or below -17.5: e^s < 2.6e-8 < 2^-24
    with torch.no_grad():
        m.entity_embedding.mul_(k)
        m.relation_embedding.mul_(k)
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    assert float(O.score(name, ent, rel, pos, neg, mode, 0.0).max()) < -17.0
    e = ent.clone().requires_grad_(True)
    r = rel.clone().requires_grad_(True)
    ref = O.tf_train_loss(name, e, r, pos, neg, w.double(), torch.tensor([mode] * B), 0.0)
    ref.backward()
    ge = e.grad[e.grad != 0].abs()
    eps = float(ge.median())
    assert eps < 1e-9  # the candidate rows' gradients are of the e^s scale
    opt = Adam(m.parameters(), lr=lr, eps=eps)
    loss = float(m.train_step_fused(pos.to(DEV), neg.to(DEV), w.to(DEV), mode, opt))
    assert abs(loss - ref.item()) <= TOL * max(1.0, abs(ref.item())), (loss, ref.item())
    for p_got, p0, gr in ((m.entity_embedding, ent, e.grad), (m.relation_embedding, rel, r.grad)):
        p1, _, _ = O.keras_adam_step(p0, gr, torch.zeros_like(p0), torch.zeros_like(p0), 1, lr, epsilon=eps)
        assert (p_got.detach().cpu().double() - p1).abs().max().item() <= 5e-2 * lr
