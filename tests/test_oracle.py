"""CPU tests of the oracle itself: the torch op-graph restatement vs the independent scalar-loop
restatement, the Q2 blend vs the selected branch, gradients vs finite differences, and the
committed golden fixtures (regression)."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import kge_oracle as O
from oracle import loops as L
from tests.conftest import rel_close

FNS = ["TransE", "DistMult", "ComplEx", "RotatE", "pRotatE", "InterHT"]
MULT = {"TransE": (1, 1), "DistMult": (1, 1), "ComplEx": (2, 2), "RotatE": (2, 1), "pRotatE": (1, 1),
        "InterHT": (2, 3)}


def _case(name, d=6, E=11, R=3, B=3, N=5, seed=0, gamma=7.0):
    em, rm = MULT[name]
    ent, rel, rng = O.make_tables(E, R, em * d, rm * d, gamma, d, seed=seed, dtype=torch.float64)
    g = np.random.RandomState(seed)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(g.randint(E, size=(B, N)))
    return ent, rel, pos, neg, gamma, rng


@pytest.mark.parametrize("name", FNS)
@pytest.mark.parametrize("mode", ["head-batch", "tail-batch", "single"])
def test_oracle_matches_scalar_loops(name, mode):
    ent, rel, pos, neg, gamma, rng = _case(name)
    mod = 0.5 * rng
    got = O.score(name, ent, rel, pos, neg, mode, gamma, rng, mod).numpy()
    ref = L.score_batch(name, ent.tolist(), rel.tolist(), pos.tolist(), neg.tolist(), mode, gamma, rng, mod)
    np.testing.assert_allclose(got, np.array(ref), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("name", ["InterHT", "RotatE", "TransE"])
def test_tf_blend_equals_selected_branch(name):
    ent, rel, pos, neg, gamma, rng = _case(name)
    for mode in (0, 1, 2, 3):  # Q1: 2 falls into tail-batch
        a = O.tf_call(name, ent, rel, pos, neg, mode, gamma, rng)
        b = O.tf_call_useful(name, ent, rel, pos, neg, mode, gamma, rng)
        assert a.shape == (pos.shape[0], 1)
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=0, atol=1e-14)


def test_adv_reduce_matches_loops():
    s = torch.from_numpy(np.random.RandomState(0).normal(scale=5.0, size=(4, 9)))
    got = O.adv_reduce(s).numpy()[:, 0]
    ref = [L.adv_reduce_row(row) for row in s.tolist()]
    np.testing.assert_allclose(got, ref, rtol=1e-12)


def test_train_loss_gradient_finite_difference():
    ent, rel, pos, neg, gamma, rng = _case("InterHT", d=4, E=7, R=2, B=2, N=3)
    w = torch.tensor([[0.5], [1.0]], dtype=torch.float64)
    e = ent.clone().requires_grad_(True)
    r = rel.clone().requires_grad_(True)
    loss = O.tf_train_loss("InterHT", e, r, pos, neg, w, torch.tensor([1]), gamma, rng)
    loss.backward()
    eps = 1e-6
    for (i, j) in [(int(pos[0, 0]), 1), (int(neg[1, 2]), 5), (int(pos[1, 2]), 0)]:
        ep = ent.clone(); ep[i, j] += eps
        em = ent.clone(); em[i, j] -= eps
        fd = (O.tf_train_loss("InterHT", ep, rel, pos, neg, w, torch.tensor([1]), gamma, rng)
              - O.tf_train_loss("InterHT", em, rel, pos, neg, w, torch.tensor([1]), gamma, rng)) / (2 * eps)
        assert abs(float(fd) - float(e.grad[i, j])) < 1e-6


def test_tf_dims_q5():
    # -dr is dead (model.py:65-78): relation_dim = hidden without -tr, 3*hidden with -tr
    assert O.tf_dims("InterHT", 10, de=True, dr=True, tr=False) == (20, 10)
    assert O.tf_dims("InterHT", 10, de=True, dr=True, tr=True) == (20, 30)
    assert O.tf_dims("TransE", 10, de=False, dr=True) == (10, 10)


def test_init_range_q8():
    ent, rel, rng = O.make_tables(50, 4, 20, 30, 24.0, 10)
    assert abs(rng - 2.6) < 1e-6
    assert float(ent.abs().max()) <= rng and float(rel.abs().max()) <= rng


GOLDEN_FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


def test_golden_files_present():
    assert len(GOLDEN_FILES) >= 20


@pytest.mark.parametrize("path", [p for p in GOLDEN_FILES if os.path.basename(p).startswith(("rand_", "c1_", "c2_"))],
                         ids=os.path.basename)
def test_oracle_reproduces_golden_scores(path):
    z = np.load(path)
    base = os.path.basename(path)
    name = "TransE" if base.startswith("c1_") else ("InterHT" if base.startswith("c2_") else base.split("_")[1])
    ent = torch.from_numpy(z["ent"]).double()
    rel = torch.from_numpy(z["rel"]).double()
    pos, neg = torch.from_numpy(z["pos"]), torch.from_numpy(z["neg"])
    for mode, tag in ((0, "head"), (1, "tail"), (3, "single")):
        got = O.score(name, ent, rel, pos, neg, mode, float(z["gamma"]), float(z["embedding_range"]),
                      float(z["modulus"])).numpy()
        assert rel_close(got, z[f"score_{tag}"], 1e-12) < 1e-12


@pytest.mark.parametrize("path", [p for p in GOLDEN_FILES if os.path.basename(p).startswith("train_")],
                         ids=os.path.basename)
def test_oracle_reproduces_golden_train(path):
    z = np.load(path)
    name = os.path.basename(path).split("_")[1]
    for mode in (0, 1):
        e = torch.from_numpy(z["ent"]).double().requires_grad_(True)
        r = torch.from_numpy(z["rel"]).double().requires_grad_(True)
        rng = float(z["embedding_range"])
        loss = O.tf_train_loss(name, e, r, torch.from_numpy(z["pos"]), torch.from_numpy(z["neg"]),
                               torch.from_numpy(z["weight"]), torch.tensor([mode]), float(z["gamma"]), rng, 0.5 * rng)
        loss.backward()
        np.testing.assert_allclose(loss.detach().numpy(), z[f"loss_mode{mode}"], rtol=1e-12)
        np.testing.assert_allclose(e.grad.numpy(), z[f"d_ent_mode{mode}"], rtol=1e-10, atol=1e-14)
        np.testing.assert_allclose(r.grad.numpy(), z[f"d_rel_mode{mode}"], rtol=1e-10, atol=1e-14)


@pytest.mark.parametrize("name", ["DistMult", "ComplEx"])
@pytest.mark.parametrize("mode", ["head-batch", "tail-batch"])
def test_dense_ranks_equal_loop_ranks(name, mode):
    """eval_ranks_dense (S = Q . ent^T at once, the C5 GPU test's checker) gives the ranks of eval_ranks (the
    per-query restatement of upstream test_step), and those ranks lie inside its [lo, hi] bounds."""
    E, R, d = 97, 5, 12
    de = name == "ComplEx"
    ent, rel, rng = O.make_tables(E, R, 2 * d if de else d, 2 * d if de else d, 24.0, d, seed=3)
    ent, rel = ent.double(), rel.double()
    g = np.random.RandomState(1)
    true = np.stack([g.randint(E, size=400), g.randint(R, size=400), g.randint(E, size=400)], 1)
    q = torch.from_numpy(true[:25])
    want = O.eval_ranks(name, ent, rel, q, mode, true, 24.0, rng)
    got, lo, hi = O.eval_ranks_dense(name, ent, rel, q, mode, true)
    assert torch.equal(got, want)
    assert bool((lo <= got).all() and (got <= hi).all())
    assert int(want.max()) > 5  # the filter and the ranks are not trivial
