"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle and the committed
golden fixtures. Tolerance for fp32 scores (north star): |got - ref| <= 1e-4 * max(1, |ref|)
against the fp64 oracle evaluated on the same fp32 inputs; indices/shapes exact."""
import glob
import os
import types

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd import ops
from customknowledgegraphembedding_amd._lib import FN_IDS
from oracle import kge_oracle as O
from tests.conftest import rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4
GOLD = os.path.join(os.path.dirname(__file__), "golden")
MULT = {"TransE": (1, 1), "DistMult": (1, 1), "ComplEx": (2, 2), "RotatE": (2, 1), "pRotatE": (1, 1),
        "InterHT": (2, 3)}
FNS = list(MULT)


def _rel_off(name, D):
    return D if name == "InterHT" else 0


def _D(name, ent_w):
    return ent_w // 2 if name in ("ComplEx", "RotatE", "InterHT") else ent_w


def _hip_scores(name, z, mode):
    ent = torch.from_numpy(z["ent"]).to(DEV)
    rel = torch.from_numpy(z["rel"]).to(DEV)
    pos = torch.from_numpy(z["pos"]).to(DEV)
    neg = torch.from_numpy(z["neg"]).to(DEV)
    D = _D(name, ent.shape[1])
    out = ops.score_indexed_raw(FN_IDS[name], mode, ent, rel, _rel_off(name, D), pos, neg, D,
                                float(z["gamma"]), float(z["embedding_range"]), float(z["modulus"]))
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _golden(prefix):
    return sorted(glob.glob(os.path.join(GOLD, prefix + "*.npz")))


def _name_of(path):
    b = os.path.basename(path)
    if b.startswith("c1_"):
        return "TransE"
    if b.startswith("c2_"):
        return "InterHT"
    return b.split("_")[1]


@pytest.mark.parametrize("path", _golden("rand_") + _golden("c1_") + _golden("c2_"), ids=os.path.basename)
def test_indexed_scores_match_golden(path):
    z = np.load(path)
    name = _name_of(path)
    for mode, tag in ((0, "head"), (1, "tail"), (3, "single")):
        got = _hip_scores(name, z, mode)
        ref = z[f"score_{tag}"]
        assert got.shape == ref.shape
        assert rel_close(got, ref) <= TOL, (name, tag, rel_close(got, ref))


@pytest.mark.parametrize("path", _golden("rand_"), ids=os.path.basename)
def test_dense_plugin_matches_golden(path):
    """model_func(head, relation, tail, mode) on rows gathered by the test (model.py:109-112)."""
    z = np.load(path)
    name = _name_of(path)
    ent = torch.from_numpy(z["ent"]).to(DEV)
    rel = torch.from_numpy(z["rel"]).to(DEV)
    pos = torch.from_numpy(z["pos"]).to(DEV)
    neg = torch.from_numpy(z["neg"]).to(DEV)
    D = _D(name, ent.shape[1])
    for mode, tag in ((0, "head"), (1, "tail"), (3, "single")):
        h, r, t = O.gather_rows(ent, rel, pos, neg, mode)
        got = ops.score_dense_raw(FN_IDS[name], mode, h, r, t, _rel_off(name, D), D, float(z["gamma"]),
                                  float(z["embedding_range"]), float(z["modulus"])).cpu().numpy()
        assert rel_close(got, z[f"score_{tag}"]) <= TOL


@pytest.mark.parametrize("path", _golden("rand_"), ids=os.path.basename)
def test_reductions_match_golden(path):
    z = np.load(path)
    s = torch.from_numpy(z["score_tail"]).float().to(DEV)
    adv = ops.neg_reduce_raw(s, 1.0, True).cpu().numpy()
    mean = ops.neg_reduce_raw(s, 1.0, False).cpu().numpy()
    assert rel_close(adv, z["adv_reduce_tail"][:, 0]) <= TOL
    assert rel_close(mean, z["mean_reduce_tail"][:, 0]) <= TOL
    ls = ops.log_sigmoid_raw(s).cpu()
    assert rel_close(ls.numpy(), F.logsigmoid(s.cpu().double()).numpy()) <= 1e-6


def _rand_case(name, D, E=300, R=9, B=5, N=37, seed=0, gamma=11.0):
    em, rm = MULT[name]
    ent, rel, rng = O.make_tables(E, R, em * D, rm * D, gamma, D, seed=seed)
    g = np.random.RandomState(seed)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(g.randint(E, size=(B, N)))
    return ent, rel, pos, neg, gamma, rng


@pytest.mark.parametrize("name", FNS)
@pytest.mark.parametrize("D", [1, 3, 50, 63, 65, 130, 257, 500, 1000, 2048])
def test_odd_and_max_dims(name, D):
    """Every vector width (16/8/4-B rows), partial groups past D, and the largest D per width."""
    if D > 512 and D % 4:
        pytest.skip("scalar rows are register-resident only up to 512")
    ent, rel, pos, neg, gamma, rng = _rand_case(name, D, seed=D)
    mod = 0.5 * rng
    for mode in (0, 1, 3):
        ref = O.score(name, ent.double(), rel.double(), pos, neg, mode, gamma, rng, mod).numpy()
        got = ops.score_indexed_raw(FN_IDS[name], mode, ent.to(DEV), rel.to(DEV), _rel_off(name, D), pos.to(DEV),
                                    neg.to(DEV), D, gamma, rng, mod).cpu().numpy()
        assert rel_close(got, ref) <= TOL, (name, D, mode, rel_close(got, ref))


@pytest.mark.parametrize("name", FNS)
def test_out_of_range_index_reads_zero_row(name):
    """TF's GPU tf.gather zero-fills out-of-range ids (model.py:130-185); so do the kernels."""
    D = 16
    ent, rel, pos, neg, gamma, rng = _rand_case(name, D, E=40, B=3, N=6)
    bad = neg.clone()
    bad[0, 1] = 40       # == nentity
    bad[1, 2] = -3       # negative
    bad[2, 5] = 10 ** 9  # far away
    ent_z = torch.cat([ent, torch.zeros(1, ent.shape[1])])   # row 40 = zeros
    ref_neg = bad.clone()
    ref_neg[(bad < 0) | (bad >= 40)] = 40
    with np.errstate(all="ignore"):
        ref = O.score(name, ent_z.double(), rel.double(), pos, ref_neg, 1, gamma, rng, 0.5 * rng).numpy()
    got = ops.score_indexed_raw(FN_IDS[name], 1, ent.to(DEV), rel.to(DEV), _rel_off(name, D), pos.to(DEV),
                                bad.to(DEV), D, gamma, rng, 0.5 * rng).cpu().numpy()
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))  # InterHT: 0/0 (Q7) -> NaN, as TF
    ok = ~np.isnan(ref)
    assert rel_close(got[ok], ref[ok]) <= TOL


def test_empty_batch_and_empty_candidates():
    ent = torch.randn(10, 8, device=DEV)
    rel = torch.randn(2, 8, device=DEV)
    pos = torch.zeros(0, 3, dtype=torch.int64, device=DEV)
    neg = torch.zeros(0, 4, dtype=torch.int64, device=DEV)
    out = ops.score_indexed_raw(0, 1, ent, rel, 0, pos, neg, 8, 1.0, 1.0)
    assert out.shape == (0, 4)
    pos = torch.zeros(2, 3, dtype=torch.int64, device=DEV)
    neg = torch.zeros(2, 0, dtype=torch.int64, device=DEV)
    out = ops.score_indexed_raw(0, 1, ent, rel, 0, pos, neg, 8, 1.0, 1.0)
    assert out.shape == (2, 0)


@pytest.mark.parametrize("path", _golden("c1_") + _golden("c2_"), ids=os.path.basename)
def test_tf_call_matches_oracle(path):
    """TFKGEModel.call(((pos, neg), mode)) -> [B,1] (model.py:114-205), modes 0, 1, 3."""
    z = np.load(path)
    name = _name_of(path)
    d = int(z["hidden_dim"])
    ent = torch.from_numpy(z["ent"])
    rel = torch.from_numpy(z["rel"])
    m = kge.TFKGEModel(name, ent.shape[0], rel.shape[0], d, float(z["gamma"]),
                       double_entity_embedding=(name == "InterHT"), triple_relation_embedding=(name == "InterHT"),
                       device=DEV)
    with torch.no_grad():
        m.entity_embedding.copy_(ent)
        m.relation_embedding.copy_(rel)
    pos, neg = torch.from_numpy(z["pos"]).to(DEV), torch.from_numpy(z["neg"]).to(DEV)
    for mode in (0, 1, 3):
        got = m(((pos, neg), mode)).detach().cpu().numpy()
        assert got.shape == (pos.shape[0], 1)
        assert rel_close(got, z[f"tf_call_mode{mode}"]) <= TOL


def _grad_close(got, ref, tol=TOL):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-12)
    return float(np.abs(got - ref).max() / scale) <= tol


@pytest.mark.parametrize("path", _golden("train_"), ids=os.path.basename)
def test_tf_train_step_loss_and_grads(path):
    """supervisor.py:17-25: loss of the two model calls and tape.gradient w.r.t. both tables
    (self-adversarial softmax NOT detached, Q3)."""
    z = np.load(path)
    name = _name_of(path)
    d = int(z["hidden_dim"])
    ent = torch.from_numpy(z["ent"])
    rel = torch.from_numpy(z["rel"])
    m = kge.TFKGEModel(name, ent.shape[0], rel.shape[0], d, float(z["gamma"]),
                       double_entity_embedding=MULT[name][0] == 2, double_relation_embedding=(name == "ComplEx"),
                       triple_relation_embedding=(name == "InterHT"), device=DEV)
    if name == "pRotatE":
        m.modulus.requires_grad_(False)
        with torch.no_grad():
            m.modulus.fill_(0.5 * float(z["embedding_range"]))
    pos, neg = torch.from_numpy(z["pos"]).to(DEV), torch.from_numpy(z["neg"]).to(DEV)
    w = torch.from_numpy(z["weight"]).float().to(DEV)
    for mode in (0, 1):
        with torch.no_grad():
            m.entity_embedding.copy_(ent)
            m.relation_embedding.copy_(rel)
        m.zero_grad(set_to_none=True)
        negative_score = m(((pos, neg), mode))
        positive_score = m(((pos, neg), 3))
        psl = -torch.sum(w * positive_score) / torch.sum(w)
        nsl = -torch.sum(w * negative_score) / torch.sum(w)
        loss = (psl + nsl) / 2
        loss.backward()
        assert rel_close(loss.item(), z[f"loss_mode{mode}"]) <= TOL
        assert _grad_close(m.entity_embedding.grad.cpu(), z[f"d_ent_mode{mode}"]), name
        assert _grad_close(m.relation_embedding.grad.cpu(), z[f"d_rel_mode{mode}"]), name


@pytest.mark.parametrize("name", FNS)
@pytest.mark.parametrize("mode", [0, 1, 3])
def test_dense_plugin_backward_matches_oracle_autograd(name, mode):
    D = 24
    ent, rel, pos, neg, gamma, rng = _rand_case(name, D, E=30, B=3, N=5, seed=7)
    mod = 0.5 * rng
    h, r, t = O.gather_rows(ent.double(), rel.double(), pos, neg, mode)
    h, r, t = (x.clone().requires_grad_(True) for x in (h, r, t))
    go = torch.from_numpy(np.random.RandomState(1).normal(size=(3, 1 if mode == 3 else 5)))
    (O.model_func(name, h, r, t, mode, gamma, rng, mod) * go).sum().backward()
    hg, rg, tg = (x.detach().float().to(DEV).requires_grad_(True) for x in (h, r, t))
    s = ops.score_dense(FN_IDS[name], mode, hg, rg, tg, D, gamma, rng, _rel_off(name, D), mod)
    (s * go.float().to(DEV)).sum().backward()
    for a, b in ((hg, h), (rg, r), (tg, t)):
        assert _grad_close(a.grad.cpu(), b.grad), (name, mode)


def test_upstream_kge_model_forward_and_train_step():
    torch.manual_seed(0)
    m = kge.KGEModel("RotatE", 200, 7, 32, 9.0, double_entity_embedding=True, device=DEV)
    g = np.random.RandomState(0)
    pos = torch.from_numpy(np.stack([g.randint(200, size=16), g.randint(7, size=16), g.randint(200, size=16)], 1))
    neg = torch.from_numpy(g.randint(200, size=(16, 12)))
    ent, rel = m.entity_embedding.detach().cpu().double(), m.relation_embedding.detach().cpu().double()
    rng = m._range_f
    got = m((pos.to(DEV), neg.to(DEV)), mode="tail-batch").detach().cpu().numpy()
    ref = O.score("RotatE", ent, rel, pos, neg, "tail-batch", 9.0, rng).numpy()
    assert rel_close(got, ref) <= TOL
    args = types.SimpleNamespace(negative_adversarial_sampling=True, adversarial_temperature=1.0,
                                 uni_weight=False, regularization=0.0)
    w = torch.rand(16)

    def it():
        while True:
            yield pos, neg, w, "tail-batch"

    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    itr = it()
    losses = [kge.KGEModel.train_step(m, opt, itr, args)["loss"] for _ in range(20)]
    assert losses[-1] < losses[0]


def test_c2_full_size_properties():
    """BASELINE config C2 (WN18RR InterHT d=1000 -de -tr, B=512, N=256) at full size:
    oracle parity on sampled rows, bitwise determinism, and single == tail-batch on the true tail."""
    E, R, d, B, N, gamma = 40943, 11, 1000, 512, 256, 24.0
    ent, rel, rng = O.make_tables(E, R, 2 * d, 3 * d, gamma, d, seed=0)
    g = np.random.RandomState(1)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(np.random.RandomState(2).randint(E, size=(B, N)))
    entd, reld, posd, negd = ent.to(DEV), rel.to(DEV), pos.to(DEV), neg.to(DEV)
    fn = FN_IDS["InterHT"]
    for mode in (0, 1):
        a = ops.score_indexed_raw(fn, mode, entd, reld, d, posd, negd, d, gamma, rng)
        b = ops.score_indexed_raw(fn, mode, entd, reld, d, posd, negd, d, gamma, rng)
        assert torch.equal(a, b)  # deterministic: fixed reduction order, no atomics
        rows = [0, 7, 255, 511]
        ref = O.score("InterHT", ent.double(), rel.double(), pos[rows], neg[rows], mode, gamma, rng).numpy()
        assert rel_close(a[rows].cpu().numpy(), ref) <= TOL
    single = ops.score_indexed_raw(fn, 3, entd, reld, d, posd, None, d, gamma, rng)
    tail_true = ops.score_indexed_raw(fn, 1, entd, reld, d, posd, posd[:, 2:3].contiguous(), d, gamma, rng)
    assert torch.equal(single, tail_true)


@pytest.mark.parametrize("path", _golden("c1_") + _golden("c2_"), ids=os.path.basename)
def test_fused_step_forward_matches_both_calls(path):
    """kge_step_forward == (call(((pos,neg),mode)), call(((pos,neg),3))) (supervisor.py:17-18)."""
    z = np.load(path)
    name = _name_of(path)
    d = int(z["hidden_dim"])
    ent = torch.from_numpy(z["ent"])
    rel = torch.from_numpy(z["rel"])
    m = kge.TFKGEModel(name, ent.shape[0], rel.shape[0], d, float(z["gamma"]),
                       double_entity_embedding=(name == "InterHT"), triple_relation_embedding=(name == "InterHT"),
                       device=DEV)
    with torch.no_grad():
        m.entity_embedding.copy_(ent)
        m.relation_embedding.copy_(rel)
    pos, neg = torch.from_numpy(z["pos"]).to(DEV), torch.from_numpy(z["neg"]).to(DEV)
    for mode in (0, 1):
        n, p = m.step_forward(pos, neg, mode)
        assert rel_close(n.detach().cpu().numpy(), z[f"tf_call_mode{mode}"]) <= TOL
        assert rel_close(p.detach().cpu().numpy(), z["tf_call_mode3"]) <= TOL
        # and bitwise identical to the unfused calls
        assert torch.equal(n, m(((pos, neg), mode)))
        assert torch.equal(p, m(((pos, neg), 3)))


@pytest.mark.parametrize("path", _golden("train_"), ids=os.path.basename)
def test_fused_step_train_grads(path):
    """Loss + tape.gradient of supervisor.py:17-25 through the fused step_forward."""
    z = np.load(path)
    name = _name_of(path)
    d = int(z["hidden_dim"])
    ent = torch.from_numpy(z["ent"])
    rel = torch.from_numpy(z["rel"])
    m = kge.TFKGEModel(name, ent.shape[0], rel.shape[0], d, float(z["gamma"]),
                       double_entity_embedding=MULT[name][0] == 2, double_relation_embedding=(name == "ComplEx"),
                       triple_relation_embedding=(name == "InterHT"), device=DEV)
    if name == "pRotatE":
        m.modulus.requires_grad_(False)
        with torch.no_grad():
            m.modulus.fill_(0.5 * float(z["embedding_range"]))
    pos, neg = torch.from_numpy(z["pos"]).to(DEV), torch.from_numpy(z["neg"]).to(DEV)
    w = torch.from_numpy(z["weight"]).float().to(DEV)
    for mode in (0, 1):
        with torch.no_grad():
            m.entity_embedding.copy_(ent)
            m.relation_embedding.copy_(rel)
        m.zero_grad(set_to_none=True)
        negative_score, positive_score = m.step_forward(pos, neg, mode)
        loss = (-torch.sum(w * positive_score) / torch.sum(w) - torch.sum(w * negative_score) / torch.sum(w)) / 2
        loss.backward()
        assert rel_close(loss.item(), z[f"loss_mode{mode}"]) <= TOL
        assert _grad_close(m.entity_embedding.grad.cpu(), z[f"d_ent_mode{mode}"]), name
        assert _grad_close(m.relation_embedding.grad.cpu(), z[f"d_rel_mode{mode}"]), name


@pytest.mark.parametrize("name", FNS)
@pytest.mark.parametrize("N", [1, 3, 67, 1030])
def test_fused_step_kernel_any_n(name, N):
    """The fused step kernel (block per batch row, four waves splitting the row's N negatives, wave 0
    finishing the row) equals the separate scoring + reduction + positive calls bitwise for N that
    do not split evenly over the waves, including N < 4 and more than 256 per wave."""
    em, rm = MULT[name]
    E, R, d, B = 300, 5, 24, 7
    m = kge.TFKGEModel(name, E, R, d, 9.0, double_entity_embedding=(em == 2),
                       double_relation_embedding=(name == "ComplEx"), triple_relation_embedding=(rm == 3),
                       device=DEV, seed=3)
    g = np.random.RandomState(N)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)).to(DEV)
    neg = torch.from_numpy(g.randint(E, size=(B, N))).to(DEV)
    with torch.no_grad():
        for mode in (0, 1):
            n, p = m.step_forward(pos, neg, mode)
            assert torch.equal(n, m(((pos, neg), mode)))
            assert torch.equal(p, m(((pos, neg), 3)))
