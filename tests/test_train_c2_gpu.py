"""The one-call train step (kge_train_step: supervisor.py:15-26) against the fp64 oracle AT THE WIDTH THE BENCH
TIMES IT: InterHT d = 1 000 `-de -tr` runs step_fwd_grad_kernel<V4, G4> and bwd_ent_stream_kernel's streaming
phase 2 (G % 4 == 0), which the d <= 250 oracle tests in test_train_gpu.py never reach.

* full C2: E = 40 943, R = 11, B = 512, N = 256, WN18RR positives (tests/golden/wn18rr_ids.npz), three steps in
  alternating modes. The oracle's loss is a sum over batch rows, so its gradient is accumulated over chunks of 32
  rows: each chunk's rows are restated on the sub-table of the entity rows the chunk touches (same values, ids
  remapped) and its gradient is scattered back (index_add). The selected branch only (O.tf_call_useful: tf_call's
  values whenever no branch is NaN; the x0 branches add exactly 0 to the fp64 gradient).
* E = 12 and E = 3 at d = 1 000: the entity buckets of phase 2 at their extremes (~800 events per row: the
  block-wide LDS sort; ~2 200: past its 2 048, the ordered extraction).
* RotatE d = 1 000 (C3's train step) with trained-range phases (the relation table scaled so phases reach
  +-8 pi): the fused train forward runs the hardware sin / cos, the backward libm's.

Bars: loss within 1e-4 relative, both tables within 5e-2 lr after Keras Adam (test_train_gpu.py's bars).
Reference: /root/reference/tensorflow_codes/supervisor.py:15-26, model.py:168-171,195-198,207-224."""
import os

import numpy as np
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd.optim import Adam
from customknowledgegraphembedding_amd.supervisor import Strategy, Sum, Trainer
from oracle import kge_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _oracle_step_chunked(name, ent, rel, pos, neg, w, mode, gamma, rng, chunk=32):
    """supervisor.py:17-23's loss and its fp64 gradient for both tables, accumulated over row chunks."""
    B = pos.shape[0]
    wsum = w.sum()
    g_ent = torch.zeros_like(ent)
    g_rel = torch.zeros_like(rel)
    loss = 0.0
    for r0 in range(0, B, chunk):
        p, n, ww = pos[r0:r0 + chunk], neg[r0:r0 + chunk], w[r0:r0 + chunk].reshape(-1, 1)
        c = p.shape[0]
        uids, inv = torch.unique(torch.cat([p[:, 0], p[:, 2], n.reshape(-1)]), return_inverse=True)
        p2 = p.clone()
        p2[:, 0], p2[:, 2] = inv[:c], inv[c:2 * c]
        n2 = inv[2 * c:].reshape(n.shape)
        sub = ent[uids].clone().requires_grad_(True)
        r = rel.clone().requires_grad_(True)
        ns = O.tf_call_useful(name, sub, r, p2, n2, mode, gamma, rng)
        ps = O.tf_call_useful(name, sub, r, p2, n2, 3, gamma, rng)
        lc = (-(ww * ps).sum() / wsum - (ww * ns).sum() / wsum) / 2
        lc.backward()
        g_ent.index_add_(0, uids, sub.grad)
        g_rel += r.grad
        loss += lc.item()
    return loss, g_ent, g_rel


def _run(name, m, batches, gamma, lr, chunk=32):
    """Three Trainer steps on the GPU (the one-call kge_train_step) and the oracle's three steps; returns the
    losses and the tables' worst deviation in units of lr."""
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    trainer = Trainer(Strategy(), batches, m, Adam(m.parameters(), lr=lr), Sum())
    assert trainer.fused and trainer.one_call
    it = iter(batches)
    losses = [float(trainer.train_step(it)) for _ in batches]
    st = {}
    ref_losses = []
    for t, (pos, neg, w, mode) in enumerate(batches, start=1):
        loss, ge, gr = _oracle_step_chunked(name, ent, rel, pos, neg, w.double(), int(mode[0]), gamma, m._range_f,
                                            chunk)
        ref_losses.append(loss)
        for key, gg in (("e", ge), ("r", gr)):
            p = ent if key == "e" else rel
            mm, vv = st.get(key, (torch.zeros_like(p), torch.zeros_like(p)))
            p2, mm, vv = O.keras_adam_step(p, gg, mm, vv, t, lr)
            st[key] = (mm, vv)
            if key == "e":
                ent = p2
            else:
                rel = p2
    de = (m.entity_embedding.detach().cpu().double() - ent).abs()
    dr = (m.relation_embedding.detach().cpu().double() - rel).abs()
    return losses, ref_losses, float(de.max()) / lr, float(dr.max()) / lr, int((de > 5e-2 * lr).sum())


def test_train_step_c2_full_size_vs_oracle():
    """C2 at full size: E = 40 943, d = 1 000 `-de -tr`, B = 512, N = 256, WN18RR positives; head-, tail-, head-
    batch steps. Loss within 1e-4, both tables within 5e-2 lr of the oracle's fp64 step + Keras Adam."""
    name, E, R, d, B, N, gamma, lr = "InterHT", 40943, 11, 1000, 512, 256, 24.0, 1e-3
    m = kge.TFKGEModel(name, E, R, d, gamma, double_entity_embedding=True, triple_relation_embedding=True,
                       device=DEV, seed=0)
    with np.load(os.path.join(GOLD, "wn18rr_ids.npz")) as z:
        tri = z["triples"].astype(np.int64)
    perm = np.random.RandomState(0).permutation(len(tri))
    batches = []
    for i in range(3):
        g = np.random.RandomState(40 + i)
        pos = torch.from_numpy(tri[perm[i * B:(i + 1) * B]])
        neg = torch.from_numpy(g.randint(E, size=(B, N)))
        w = torch.from_numpy(g.uniform(0.2, 1.0, size=(B, 1))).float()
        batches.append((pos, neg, w, torch.tensor([(i + 1) % 2] * B)))
    losses, ref, de, dr, nbad = _run(name, m, batches, gamma, lr)
    np.testing.assert_allclose(losses, ref, rtol=1e-4)
    assert de <= 5e-2 and dr <= 5e-2, (de, dr, nbad)


@pytest.mark.parametrize("E,B,N", [(12, 48, 200), (3, 40, 160)])
def test_train_step_d1000_bucket_extremes_vs_oracle(E, B, N):
    """d = 1 000 (V4 x G4) with every entity row hot: ~800 (E = 12) and ~2 200 (E = 3) events per row."""
    name, R, d, gamma, lr = "InterHT", 4, 1000, 12.0, 1e-3
    m = kge.TFKGEModel(name, E, R, d, gamma, double_entity_embedding=True, triple_relation_embedding=True,
                       device=DEV, seed=13)
    g = np.random.RandomState(6)
    batches = []
    for i in range(3):
        pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
        neg = torch.from_numpy(g.randint(E, size=(B, N)))
        w = torch.from_numpy(g.uniform(0.2, 1.0, size=(B, 1))).float()
        batches.append((pos, neg, w, torch.tensor([i % 2] * B)))
    losses, ref, de, dr, nbad = _run(name, m, batches, gamma, lr, chunk=B)
    np.testing.assert_allclose(losses, ref, rtol=1e-4)
    assert de <= 5e-2 and dr <= 5e-2, (de, dr, nbad)


@pytest.mark.parametrize("turns", [1, 4])
def test_train_step_rotate_d1000_trained_phases_vs_oracle(turns):
    """RotatE d = 1 000 `-de` (C3's train step) with the relation table scaled so the phases reach +-2 pi turns."""
    name, E, R, d, B, N, gamma, lr = "RotatE", 700, 9, 1000, 32, 256, 9.0, 1e-3
    m = kge.TFKGEModel(name, E, R, d, gamma, double_entity_embedding=True, device=DEV, seed=17)
    with torch.no_grad():
        m.relation_embedding.mul_(2.0 * turns)
    ph = float(m.relation_embedding.detach().abs().max()) / (m._range_f / np.pi)
    assert ph > 1.8 * np.pi * turns
    g = np.random.RandomState(turns)
    batches = []
    for i in range(3):
        pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
        neg = torch.from_numpy(g.randint(E, size=(B, N)))
        w = torch.from_numpy(g.uniform(0.2, 1.0, size=(B, 1))).float()
        batches.append((pos, neg, w, torch.tensor([i % 2] * B)))
    losses, ref, de, dr, nbad = _run(name, m, batches, gamma, lr, chunk=B)
    np.testing.assert_allclose(losses, ref, rtol=1e-4)
    assert de <= 5e-2 and dr <= 5e-2, (de, dr, nbad)
