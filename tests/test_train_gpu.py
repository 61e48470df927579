"""GPU tests of the train-step half of the path: the HIP Adam kernel (Keras and torch rules) and
Trainer.train_step (supervisor.py:13-30) against the oracle's TF-semantics step."""
import numpy as np
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd.optim import Adam
from customknowledgegraphembedding_amd.supervisor import Strategy, Sum, Trainer
from oracle import kge_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("n", [1, 7, 4096, 100003])
def test_adam_keras_matches_oracle(n):
    g0 = torch.Generator().manual_seed(n)
    p = torch.randn(n, generator=g0, dtype=torch.float64)
    pk = p.float().to(DEV)
    opt = Adam([torch.nn.Parameter(pk)], lr=1e-2, semantics="keras")
    param = opt.param_groups[0]["params"][0]
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for t in range(1, 4):
        g = torch.randn(n, generator=g0, dtype=torch.float64)
        param.grad = g.float().to(DEV)
        opt.step()
        p, m, v = O.keras_adam_step(p, g.float().double(), m, v, t, 1e-2)
    err = (param.detach().double().cpu() - p).abs().max().item()
    assert err <= 1e-6, err


@pytest.mark.parametrize("offset", [1, 2, 3])
def test_adam_on_unaligned_parameter_view(offset):
    """a parameter that is an offset view (4-byte, not 16-byte aligned) takes the dword
    path and gives bitwise the update of an aligned copy."""
    g0 = torch.Generator().manual_seed(offset)
    base = torch.randn(4099 + offset, generator=g0).to(DEV)
    view = torch.nn.Parameter(base[offset:])  # shares storage at a 4*offset-byte offset
    assert view.data_ptr() % 16 != 0
    ref = torch.nn.Parameter(base[offset:].clone())
    o1, o2 = Adam([view], lr=1e-2), Adam([ref], lr=1e-2)
    for _ in range(3):
        gr = torch.randn(4099, generator=g0).to(DEV)
        view.grad, ref.grad = gr.clone(), gr.clone()
        o1.step()
        o2.step()
    assert torch.equal(view.detach(), ref.detach())
    assert o1.state[view]["step"] == 3


def test_adam_torch_semantics_matches_torch_optim():
    torch.manual_seed(0)
    a = torch.nn.Parameter(torch.randn(5000, device=DEV))
    b = torch.nn.Parameter(a.detach().clone())
    o1 = Adam([a], lr=3e-3, semantics="torch")
    o2 = torch.optim.Adam([b], lr=3e-3, foreach=False)
    for _ in range(4):
        g = torch.randn(5000, device=DEV)
        a.grad = g.clone()
        b.grad = g.clone()
        o1.step()
        o2.step()
    assert (a - b).abs().max().item() <= 1e-6


def test_trainer_train_step_matches_oracle_tf_step():
    """Three Trainer.train_step calls (HIP forward, backward, Keras Adam) vs the oracle: TF loss
    graph in fp64 autograd + Keras Adam, same data, same lr."""
    name, E, R, d, B, N, gamma, lr = "InterHT", 60, 4, 16, 6, 8, 12.0, 1e-3
    m = kge.TFKGEModel(name, E, R, d, gamma, double_entity_embedding=True, triple_relation_embedding=True,
                       device=DEV, seed=11)
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    g = np.random.RandomState(4)
    batches = []
    for i in range(3):
        pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
        neg = torch.from_numpy(g.randint(E, size=(B, N)))
        w = torch.from_numpy(g.uniform(0.2, 1.0, size=(B, 1))).float()
        batches.append((pos, neg, w, torch.tensor([i % 2] * B)))
    trainer = Trainer(Strategy(), batches, m, Adam(m.parameters(), lr=lr), Sum())
    it = iter(batches)
    losses = [float(trainer.train_step(it)) for _ in range(3)]

    st = {}
    ref_losses = []
    for t, (pos, neg, w, mode) in enumerate(batches, start=1):
        e = ent.clone().requires_grad_(True)
        r = rel.clone().requires_grad_(True)
        loss = O.tf_train_loss(name, e, r, pos, neg, w.double(), mode, gamma, m._range_f)
        loss.backward()
        ref_losses.append(loss.item())
        for key, p, gr in (("e", ent, e.grad), ("r", rel, r.grad)):
            mm, vv = st.get(key, (torch.zeros_like(p), torch.zeros_like(p)))
            p2, mm, vv = O.keras_adam_step(p, gr, mm, vv, t, lr)
            st[key] = (mm, vv)
            if key == "e":
                ent = p2.detach()
            else:
                rel = p2.detach()
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-4)
    # Adam's m/sqrt(v) amplifies fp32-vs-fp64 differences only where |g| ~ eps; bound by lr
    assert (m.entity_embedding.detach().cpu().double() - ent).abs().max().item() <= 5e-2 * lr
    assert (m.relation_embedding.detach().cpu().double() - rel).abs().max().item() <= 5e-2 * lr
    assert float(trainer.metrics.result()) == pytest.approx(losses[-1] + losses[0] + losses[1], rel=1e-5)


@pytest.mark.parametrize("name", ["InterHT", "TransE", "DistMult", "ComplEx", "RotatE", "pRotatE"])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("d", [40, 800, 1500])
def test_step_backward_deterministic_and_matches_atomic_path(name, mode, d):
    """kge_step_backward (two-phase, no float atomics) is bitwise reproducible and equals the
    atomic-scatter backward of the unfused calls to fp32 rounding, including hot entities that
    collect many events (a small table: > 64 events per row exercises the large-bucket path).
    d = 40 runs the register-resident phases; 800 and 1500 the streaming ones (1 and 2 column groups
    per wave)."""
    cfg = {"InterHT": (True, False, True), "TransE": (False, False, False), "DistMult": (False, False, False),
           "ComplEx": (True, True, False), "RotatE": (True, False, False), "pRotatE": (False, False, False)}
    de, dr, tr = cfg[name]
    E, R, B, N = 50, 3, 64, 96
    m = kge.TFKGEModel(name, E, R, d, 8.0, de, dr, tr, device=DEV, seed=9)
    g = np.random.RandomState(mode)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)).to(DEV)
    neg = torch.from_numpy(g.randint(E, size=(B, N))).to(DEV)
    w = torch.from_numpy(g.uniform(0.1, 1, size=(B, 1))).float().to(DEV)

    def grads(fused):
        m.zero_grad(set_to_none=True)
        if fused:
            n_s, p_s = m.step_forward(pos, neg, mode)
        else:
            n_s, p_s = m(((pos, neg), mode)), m(((pos, neg), 3))
        loss = (-(w * p_s).sum() - (w * n_s).sum()) / (2 * w.sum())
        loss.backward()
        out = [m.entity_embedding.grad.clone(), m.relation_embedding.grad.clone()]
        if name == "pRotatE":
            out.append(m.modulus.grad.clone())
        return out

    a = grads(True)
    b = grads(True)
    c = grads(False)
    for x, y, z in zip(a, b, c):
        assert torch.equal(x, y)  # bitwise reproducible
        scale = float(z.abs().max().clamp_min(1e-12))
        assert float((x - z).abs().max()) <= 1e-5 * scale + 1e-7, name


@pytest.mark.parametrize("name", ["InterHT", "DistMult", "RotatE", "pRotatE"])
@pytest.mark.parametrize("semantics", ["keras", "torch"])
@pytest.mark.parametrize("d", [32, 1000])
def test_fused_train_step_equals_autograd_path(name, semantics, d):
    """Trainer with the optimizer fused into the backward (kge_step_backward_adam) leaves tables,
    Adam moments and losses bitwise equal to the autograd path (kge_step_backward + kge_adam_update)."""
    cfg = {"InterHT": (True, False, True), "DistMult": (False, False, False), "RotatE": (True, False, False),
           "pRotatE": (False, False, False)}
    de, dr, tr = cfg[name]
    E, R, B, N = 300, 6, 48, 40

    def make():
        return kge.TFKGEModel(name, E, R, d, 10.0, de, dr, tr, device=DEV, seed=21)

    g = np.random.RandomState(3)
    data = []
    for i in range(4):
        pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
        neg = torch.from_numpy(g.randint(E, size=(B, N)))
        w = torch.from_numpy(g.uniform(0.1, 1, size=(B, 1))).float()
        data.append((pos, neg, w, torch.tensor([i % 2] * B)))
    runs = []
    for fused in ("split", False):
        m = make()
        opt = Adam(m.parameters(), lr=2e-3, semantics=semantics)
        tr_ = Trainer(Strategy(), data, m, opt, Sum(), fused=fused)
        assert tr_.fused == bool(fused)
        it = iter(data)
        losses = [float(tr_.train_step(it)) for _ in range(4)]
        trainable = [p for p in m.parameters() if p.requires_grad]
        runs.append((losses, [p.detach().clone() for p in trainable],
                     [opt.state[p]["exp_avg_sq"].clone() for p in trainable]))
    (la, pa, va), (lb, pb, vb) = runs
    assert la == lb
    for x, y in zip(pa + va, pb + vb):
        assert torch.equal(x, y)


@pytest.mark.parametrize("name", ["InterHT", "TransE", "DistMult", "ComplEx", "RotatE"])
@pytest.mark.parametrize("d", [24, 250, 1000, 1500])
def test_one_call_train_step_matches_split_path(name, d):
    """kge_train_step (phase 1 fused into the forward, online-softmax running sums, event bucketing on
    a side stream) against the split path (kge_step_forward + kge_step_loss + kge_step_backward_adam):
    same losses to fp32 rounding, tables and Adam moments within a small multiple of lr, bitwise
    reproducible run to run. Head- and tail-batch steps alternate; d = 1500 takes the fallback (separate
    phase 1); hot entities (E small) exercise the large event buckets."""
    cfg = {"InterHT": (True, False, True), "TransE": (False, False, False), "DistMult": (False, False, False),
           "ComplEx": (True, True, False), "RotatE": (True, False, False)}
    de, dr, tr = cfg[name]
    E, R, B, N, lr = 90, 5, 40, 72, 2e-3
    g = np.random.RandomState(8)
    data = []
    for i in range(4):
        pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
        neg = torch.from_numpy(g.randint(E, size=(B, N)))
        w = torch.from_numpy(g.uniform(0.1, 1, size=(B, 1))).float()
        data.append((pos, neg, w, torch.tensor([i % 2] * B)))

    def run(fused):
        m = kge.TFKGEModel(name, E, R, d, 9.0, de, dr, tr, device=DEV, seed=5)
        opt = Adam(m.parameters(), lr=lr)
        tr_ = Trainer(Strategy(), data, m, opt, Sum(), fused=fused)
        it = iter(data)
        losses = [float(tr_.train_step(it)) for _ in range(4)]
        ps = [p.detach().clone() for p in m.parameters() if p.requires_grad]
        ms = [opt.state[p]["exp_avg"].clone() for p in m.parameters() if p.requires_grad]
        return losses, ps, ms

    la, pa, ma = run(True)
    lb, pb, mb = run(True)
    lc, pc, mc = run("split")
    assert la == lb
    for x, y in zip(pa + ma, pb + mb):
        assert torch.equal(x, y)  # deterministic
    np.testing.assert_allclose(la, lc, rtol=2e-6, atol=1e-7)
    for x, y in zip(pa, pc):
        # Adam's m / sqrt(v) amplifies rounding-level gradient differences only where |g| ~ eps
        assert float((x - y).abs().max()) <= 2e-2 * lr, name
    for x, y in zip(ma, mc):
        scale = float(y.abs().max().clamp_min(1e-12))
        assert float((x - y).abs().max()) <= 1e-4 * scale, name


@pytest.mark.parametrize("name", ["InterHT", "DistMult"])
def test_one_call_train_step_matches_split_path_many_events(name):
    """B·N + 3B = 300 900 events: past one round of the epilogue's scatter blocks (at most 256 blocks × 256
    threads × 4 codes = 262 144 per round), so the scatter loops and every bucket is still filled exactly once."""
    de, tr = (True, True) if name == "InterHT" else (False, False)
    E, R, B, N, d, lr = 4000, 5, 300, 1000, 24, 2e-3
    g = np.random.RandomState(21)
    data = []
    for i in range(2):
        pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
        neg = torch.from_numpy(g.randint(E, size=(B, N)))
        w = torch.from_numpy(g.uniform(0.1, 1, size=(B, 1))).float()
        data.append((pos, neg, w, torch.tensor([i % 2] * B)))

    def run(fused):
        m = kge.TFKGEModel(name, E, R, d, 9.0, de, False, tr, device=DEV, seed=5)
        opt = Adam(m.parameters(), lr=lr)
        tr_ = Trainer(Strategy(), data, m, opt, Sum(), fused=fused)
        it = iter(data)
        losses = [float(tr_.train_step(it)) for _ in range(2)]
        return losses, [p.detach().clone() for p in m.parameters() if p.requires_grad]

    la, pa = run(True)
    lc, pc = run("split")
    np.testing.assert_allclose(la, lc, rtol=2e-6, atol=1e-7)
    for x, y in zip(pa, pc):
        assert float((x - y).abs().max()) <= 2e-2 * lr, name


@pytest.mark.parametrize("E,B,N", [(60, 6, 24), (12, 48, 200), (3, 40, 160)])
def test_one_call_train_step_matches_oracle_tf_step(E, B, N):
    """kge_train_step against the oracle's fp64 TF-semantics step (loss graph + Keras Adam). E = 12 puts
    ~800 events in each entity bucket (phase 2's block-wide LDS sort), E = 3 ~2 200 (past the sort's 2 048:
    the ordered-extraction fallback)."""
    name, R, d, gamma, lr = "InterHT", 4, 200, 12.0, 1e-3
    m = kge.TFKGEModel(name, E, R, d, gamma, double_entity_embedding=True, triple_relation_embedding=True,
                       device=DEV, seed=13)
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    g = np.random.RandomState(6)
    batches = []
    for i in range(3):
        pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
        neg = torch.from_numpy(g.randint(E, size=(B, N)))
        w = torch.from_numpy(g.uniform(0.2, 1.0, size=(B, 1))).float()
        batches.append((pos, neg, w, torch.tensor([i % 2] * B)))
    trainer = Trainer(Strategy(), batches, m, Adam(m.parameters(), lr=lr), Sum())
    assert trainer.fused and trainer.one_call
    it = iter(batches)
    losses = [float(trainer.train_step(it)) for _ in range(3)]
    st = {}
    ref_losses = []
    for t, (pos, neg, w, mode) in enumerate(batches, start=1):
        e = ent.clone().requires_grad_(True)
        r = rel.clone().requires_grad_(True)
        loss = O.tf_train_loss(name, e, r, pos, neg, w.double(), mode, gamma, m._range_f)
        loss.backward()
        ref_losses.append(loss.item())
        for key, p, gr in (("e", ent, e.grad), ("r", rel, r.grad)):
            mm, vv = st.get(key, (torch.zeros_like(p), torch.zeros_like(p)))
            p2, mm, vv = O.keras_adam_step(p, gr, mm, vv, t, lr)
            st[key] = (mm, vv)
            if key == "e":
                ent = p2.detach()
            else:
                rel = p2.detach()
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-4)
    assert (m.entity_embedding.detach().cpu().double() - ent).abs().max().item() <= 5e-2 * lr
    assert (m.relation_embedding.detach().cpu().double() - rel).abs().max().item() <= 5e-2 * lr


def _twin_step(name, E, R, d, B, N, ws_fill, shapes):
    """Run `shapes` (a list of (B, N)) train steps on one model whose workspace starts filled with
    `ws_fill` bytes, and the same steps on fresh models with fresh zero workspaces; return both."""
    from customknowledgegraphembedding_amd import _lib
    g = np.random.RandomState(12)
    data = []
    for i, (b, n) in enumerate(shapes):
        pos = torch.from_numpy(np.stack([g.randint(E, size=b), g.randint(R, size=b), g.randint(E, size=b)], 1))
        neg = torch.from_numpy(g.randint(E, size=(b, n)))
        w = torch.from_numpy(g.uniform(0.1, 1.0, size=(b,))).float()
        data.append((pos.to(DEV), neg.to(DEV), w.to(DEV), i % 2))
    a = kge.TFKGEModel(name, E, R, d, 9.0, True, False, True, device=DEV, seed=3)
    oa = Adam(a.parameters(), lr=1e-3)
    nbytes = max(_lib.load().kge_train_step_workspace_size(4, E, R, a.relation_embedding.stride(0), b, n, d)
                 for b, n in shapes)
    a._train_ws = torch.full((nbytes,), ws_fill, dtype=torch.uint8, device=DEV)
    b_ = kge.TFKGEModel(name, E, R, d, 9.0, True, False, True, device=DEV, seed=3)
    ob = Adam(b_.parameters(), lr=1e-3)
    la, lb = [], []
    for pos, neg, w, mode in data:
        la.append(float(a.train_step_fused(pos, neg, w, mode, oa)))
        b_._train_ws = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)  # fresh every step
        lb.append(float(b_.train_step_fused(pos, neg, w, mode, ob)))
    return (la, list(a.parameters())), (lb, list(b_.parameters()))


@pytest.mark.parametrize("fill", [0x7F, 0xFF, 0x01])
def test_train_step_garbage_workspace_gives_correct_first_step(fill):
    """kge_train_step keeps no state in its workspace: a workspace filled with garbage (counters
    0x7F7F7F7F, -1, 0x01010101) gives bitwise the same first step as a zero-filled one."""
    (la, pa), (lb, pb) = _twin_step("InterHT", 70, 4, 96, 16, 24, fill, [(16, 24), (16, 24)])
    assert la == lb
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)


def test_train_step_workspace_reused_at_a_smaller_batch():
    """the cached workspace is reused when a later call has a smaller B (the count region
    then lands on the previous call's float data); the step must still equal a fresh-workspace step."""
    (la, pa), (lb, pb) = _twin_step("InterHT", 70, 4, 96, 16, 24, 0,
                                    [(16, 24), (8, 24), (16, 12), (3, 40)])
    assert la == lb
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)


def test_rejected_train_step_does_not_advance_adam_step():
    """a call the library rejects (here: a float64 weight pointer is fine, but a
    negative-mode check fails for mode 3) must leave the optimizer's step counters unchanged."""
    m = kge.TFKGEModel("InterHT", 40, 3, 16, 9.0, True, False, True, device=DEV, seed=1)
    opt = Adam(m.parameters(), lr=1e-3)
    pos = torch.tensor([[0, 1, 2], [3, 0, 5]], device=DEV)
    neg = torch.randint(0, 40, (2, 7), device=DEV)
    w = torch.ones(2, device=DEV)
    m.train_step_fused(pos, neg, w, 1, opt)
    assert opt.state[m.entity_embedding]["step"] == 1
    with pytest.raises(Exception):
        m.train_step_fused(pos, neg, w, 3, opt)
    assert opt.state[m.entity_embedding]["step"] == 1
    assert opt.state[m.relation_embedding]["step"] == 1
