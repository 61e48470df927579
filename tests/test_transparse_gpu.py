"""TranSparse (tensorflow_codes/model.py:96-106,139-142,161-164,187-190,226-235) on the GPU: the MFMA
forward and the deterministic backward through the C-ABI against the fp64 oracle (torch autograd on
the same fp32 inputs). Scores: |got - ref| <= 1e-4 * max(1, |ref|). Gradients: |got - ref| <=
1e-4 * max|ref| per tensor (fp32 sums over up to d * N terms)."""
import numpy as np
import pytest
import torch

from customknowledgegraphembedding_amd import ops
from customknowledgegraphembedding_amd.model import TFKGEModel
from oracle import kge_oracle as O
from tests.conftest import rel_close

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tables(E, R, d, seed=0, gamma=12.0):
    g = torch.Generator().manual_seed(seed)
    rng = (gamma + 2.0) / d
    ent = torch.empty(E, d).uniform_(-rng, rng, generator=g)
    rel = torch.empty(R, d).uniform_(-rng, rng, generator=g)
    W = torch.empty(R, d, d).uniform_(-rng, rng, generator=g)
    mask = (torch.empty(R, d, d).uniform_(1, 100, generator=g) >= 50).float()
    return ent, rel, W, mask


def _batch(E, R, B, N, seed=1):
    g = np.random.RandomState(seed)
    pos = np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1).astype(np.int64)
    neg = g.randint(E, size=(B, N)).astype(np.int64)
    return torch.from_numpy(pos), torch.from_numpy(neg)


def _oracle(ent, rel, W, mask, pos, neg, mode, gamma, grad=None):
    t = [x.double().requires_grad_(True) for x in (ent, rel, W)]
    s = O.transparse_score(t[0], t[1], t[2], mask.double(), pos, neg, mode, gamma)
    if grad is None:
        return s.detach().numpy(), None
    (s * grad.double()).sum().backward()
    return s.detach().numpy(), [x.grad.numpy() for x in t]


CASES = [  # (E, R, d, B, N)
    (97, 3, 8, 4, 16),
    (61, 2, 50, 5, 7),       # d % 4 != 0: scalar loads
    (200, 5, 130, 6, 200),   # partial K/column tiles, 2 row chunks per batch row
    (300, 2, 256, 300, 3),   # > 128 batch rows per relation: grouped chunks
]


@pytest.mark.parametrize("E,R,d,B,N", CASES)
@pytest.mark.parametrize("mode", [0, 1, 3])
@pytest.mark.parametrize("premul", [False, True])
def test_forward_parity(E, R, d, B, N, mode, premul):
    gamma = 12.0
    ent, rel, W, mask = _tables(E, R, d)
    pos, neg = _batch(E, R, B, N)
    ref, _ = _oracle(ent, rel, W, mask, pos, neg, mode, gamma)
    Wd, md = W.to(DEV), mask.to(DEV)
    M = ops.transparse_premul(Wd, md) if premul and d % 4 == 0 else None
    got = ops.transparse_score_raw(mode, ent.to(DEV), rel.to(DEV), Wd, md, pos.to(DEV), neg.to(DEV), gamma, M=M)
    torch.cuda.synchronize()
    got = got.cpu().numpy()
    assert got.shape == ref.shape
    assert rel_close(got, ref) <= 1e-4


@pytest.mark.parametrize("E,R,d,B,N", CASES)
@pytest.mark.parametrize("mode", [0, 1, 3])
def test_backward_parity_and_determinism(E, R, d, B, N, mode):
    gamma = 12.0
    ent, rel, W, mask = _tables(E, R, d, seed=3)
    pos, neg = _batch(E, R, B, N, seed=4)
    Nc = N if mode == 0 else 1
    grad = torch.from_numpy(np.random.RandomState(5).randn(B, Nc).astype(np.float32))
    _, ref = _oracle(ent, rel, W, mask, pos, neg, mode, gamma, grad)
    outs = []
    for _ in range(2):
        t = [x.to(DEV).requires_grad_(True) for x in (ent, rel, W)]
        s = ops.transparse_score(mode, t[0], t[1], t[2], mask.to(DEV), pos.to(DEV), neg.to(DEV), gamma)
        s.backward(grad.to(DEV))
        torch.cuda.synchronize()
        outs.append([x.grad.cpu().numpy() for x in t])
    for name, g, r in zip(("d_ent", "d_rel", "d_W"), outs[0], ref):
        scale = max(np.abs(r).max(), 1e-30)
        assert np.abs(g - r).max() <= 1e-4 * scale, name
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)  # bitwise deterministic


def test_backward_with_premultiplied_matrices_is_identical():
    E, R, d, B, N = 200, 2, 64, 8, 40
    ent, rel, W, mask = (x.to(DEV) for x in _tables(E, R, d, seed=21))
    pos, neg = (x.to(DEV) for x in _batch(E, R, B, N, seed=22))
    g = torch.randn(B, N, device=DEV)
    st = torch.empty(B * N, 2, device=DEV)
    M = ops.transparse_premul(W, mask)
    s0 = ops.transparse_score_raw(0, ent, rel, W, mask, pos, neg, 12.0, stats=st)
    s1 = ops.transparse_score_raw(0, ent, rel, W, mask, pos, neg, 12.0, M=M)
    assert torch.equal(s0, s1)
    grads = []
    for MM in (None, M):
        d = [torch.zeros_like(ent), torch.zeros_like(rel), torch.zeros_like(W)]
        ops.transparse_score_bwd_raw(0, ent, rel, W, mask, pos, neg, st, g, *d, M=MM)
        grads.append(d)
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_out_of_range_ids_give_nan_rows():
    E, R, d, B, N = 50, 3, 16, 4, 5
    ent, rel, W, mask = _tables(E, R, d)
    pos, neg = _batch(E, R, B, N)
    neg[1, 2] = E + 5        # zero entity row -> NaN score
    pos[2, 1] = R + 1        # zero relation -> NaN row
    got = ops.transparse_score_raw(0, ent.to(DEV), rel.to(DEV), W.to(DEV), mask.to(DEV), pos.to(DEV), neg.to(DEV),
                                   12.0).cpu().numpy()
    assert np.isnan(got[1, 2]) and np.isnan(got[2]).all()
    ok = np.ones_like(got, dtype=bool)
    ok[1, 2] = False
    ok[2] = False
    assert np.isfinite(got[ok]).all()
    got1 = ops.transparse_score_raw(3, ent.to(DEV), rel.to(DEV), W.to(DEV), mask.to(DEV), pos.to(DEV), None,
                                    12.0).cpu().numpy()
    assert np.isnan(got1[2, 0]) and np.isfinite(np.delete(got1, 2, 0)).all()


def test_model_call_and_plugin_match_oracle():
    E, R, hd, B, N = 120, 4, 32, 6, 10
    m = TFKGEModel("TranSparse", E, R, hd, 12.0, device=DEV, seed=7)
    assert m.W.shape == (R, hd, hd) and 0.4 < float(m.mask.mean()) < 0.6
    pos, neg = _batch(E, R, B, N, seed=9)
    pd, nd = pos.to(DEV), neg.to(DEV)
    ent, rel, W, mask = (x.detach().cpu() for x in (m.entity_embedding, m.relation_embedding, m.W, m.mask))
    for mode in (0, 1, 3):
        got = m(((pd, nd), mode)).detach().cpu().numpy()
        ref = O.tf_call_transparse(ent.double(), rel.double(), W.double(), mask.double(), pos, neg, mode, 12.0)
        assert rel_close(got, ref.numpy()) <= 1e-4
    # model_func plugin on pre-gathered tensors (model.py:161-164)
    head = m.entity_embedding[nd]
    relation = m.relation_embedding[pd[:, 1]].unsqueeze(1)
    tail = m.entity_embedding[pd[:, 2]].unsqueeze(1)
    s = m.model_func["TranSparse"](head, relation, tail, 0, m.W[pd[:, 1]], m.mask[pd[:, 1]])
    ref = O.transparse(head.detach().cpu().double(), relation.detach().cpu().double(), None, "head-batch", 12.0,
                       W[pos[:, 1]].double(), mask[pos[:, 1]].double())
    assert rel_close(s.detach().cpu().numpy(), ref.numpy()) <= 1e-4


def test_trainer_step_matches_oracle_loss():
    from customknowledgegraphembedding_amd.optim import Adam
    from customknowledgegraphembedding_amd.supervisor import Strategy, Sum, Trainer

    E, R, hd, B, N = 90, 3, 24, 8, 12
    m = TFKGEModel("TranSparse", E, R, hd, 12.0, device=DEV, seed=11)
    ent, rel, W, mask = (x.detach().cpu().double() for x in (m.entity_embedding, m.relation_embedding, m.W, m.mask))
    pos, neg = _batch(E, R, B, N, seed=13)
    w = torch.rand(B, 1, generator=torch.Generator().manual_seed(1))
    mode = torch.zeros(B, dtype=torch.int64)
    opt = Adam([m.entity_embedding, m.relation_embedding, m.W], lr=1e-3)
    tr = Trainer(Strategy(), None, m, opt, Sum())
    assert not tr.fused
    loss = tr.train_step(iter([(pos, neg, w, mode)]))
    t = [x.clone().requires_grad_(True) for x in (ent, rel, W)]
    wd = w.double().reshape(-1, 1)
    ns = O.tf_call_transparse(t[0], t[1], t[2], mask, pos, neg, 0, 12.0)
    ps = O.tf_call_transparse(t[0], t[1], t[2], mask, pos, neg, 3, 12.0)
    ref = (-(wd * ps).sum() / wd.sum() - (wd * ns).sum() / wd.sum()) / 2
    assert abs(float(loss) - float(ref.detach())) <= 1e-5 * max(1.0, abs(float(ref.detach())))
    ref.backward()
    # one Keras Adam step from zero moments: every touched coordinate moves by ~lr * sign(g)
    for p0, prm, g in zip((ent, rel, W), (m.entity_embedding, m.relation_embedding, m.W), (t[0].grad, t[1].grad,
                                                                                            t[2].grad)):
        exp, _, _ = O.keras_adam_step(p0, g, torch.zeros_like(p0), torch.zeros_like(p0), 1, 1e-3)
        got = prm.detach().cpu().double()
        big = g.abs() > 1e-6 * float(g.abs().max())
        assert torch.allclose(got[big], exp[big], atol=1e-6)


@pytest.mark.parametrize("d,N,premul", [(500, 256, True), (500, 300, False), (128, 200, True), (260, 129, False),
                                        (1024, 160, True)])
def test_split_once_forward_is_bitwise_the_register_split_one(monkeypatch, d, N, premul):
    """ts_fwd_x3s_kernel (operands split once at staging, buffer loads; or M_r from bf16 planes split once per
    call) against ts_fwd_x3_kernel (the same products split per fragment in the MFMA loop): head-batch scores and
    stats are bitwise equal, with
    out-of-range ids, partial K chunks and partial column super-tiles; and within 1e-4 of the fp64 oracle."""
    E, R, B, gamma = 300, 3, 5, 12.0
    ent, rel, W, mask = _tables(E, R, d, seed=4)
    pos, neg = _batch(E, R, B, N, seed=9)
    neg[1, 3] = E + 7
    neg[4, N - 1] = -2
    ed, rd, Wd, md = ent.to(DEV), rel.to(DEV), W.to(DEV), mask.to(DEV)
    M = ops.transparse_premul(Wd, md) if premul else None
    outs = []
    # 1: split per fragment in registers (ts_fwd_x3_kernel); 0 + workspace: M_r split once into bf16 planes per
    # call (ts_mplanes_kernel + ts_fwd_x3s_kernel<.., true>); 0 without: split once at staging (ts_fwd_x3s_kernel)
    # 2: the split-once kernel in the compiler's instruction order (staging after the MFMAs)
    for form, split in ((1, True), (0, True), (0, False), (2, True), (2, False)):
        st = torch.empty((B * N, 2), dtype=torch.float32, device=DEV)
        s = ops.transparse_score_raw(0, ed, rd, Wd, md, pos.to(DEV), neg.to(DEV), gamma, stats=st, M=M,
                                     forms=dict(transparse_form=form), split=split)
        torch.cuda.synchronize()
        outs.append((s.cpu(), st.cpu()))
    for o in outs[1:]:
        assert np.array_equal(outs[0][0].numpy(), o[0].numpy(), equal_nan=True)
        assert np.array_equal(outs[0][1].numpy(), o[1].numpy(), equal_nan=True)
    ok = (neg >= 0) & (neg < E)
    ref, _ = _oracle(ent, rel, W, mask, pos, neg.clamp(0, E - 1), 0, gamma)
    got = outs[1][0].numpy()
    assert rel_close(got[ok.numpy()], ref[ok.numpy()]) <= 1e-4
    assert np.isnan(got[~ok.numpy()]).all()


@pytest.mark.parametrize("d,B,R,premul", [(500, 200, 3, True), (500, 130, 5, False), (1024, 70, 2, True),
                                          (516, 90, 4, False)])
@pytest.mark.parametrize("mode", [1, 3])
def test_grouped_forward_all_columns_per_block(monkeypatch, d, B, R, premul, mode):
    """Single / tail-batch rows: one relation's row chunk per block over all columns (ts_fwd_x3g_kernel<8, 2>),
    and split over 128-column x 128-k ranges through a workspace (ts_fwd_x3g_kernel<4, 1, 2, MASK> + the ordered
    finish ts_xk_finish_kernel):
    within 1e-4 of the fp64 oracle, within fp32 rounding of ts_rows_kernel's column order (form 1) and of each
    other, bitwise run to run, with rows of out-of-range relations and heads (NaN), more than 64 rows per
    relation and d past one 512-column pass."""
    E, gamma = 400, 12.0
    ent, rel, W, mask = _tables(E, R, d, seed=5)
    pos, neg = _batch(E, R, B, 3, seed=11)
    pos[3, 1] = R + 2   # zero relation row -> NaN
    pos[5, 0] = E + 1   # zero head row -> NaN
    ed, rd, Wd, md = ent.to(DEV), rel.to(DEV), W.to(DEV), mask.to(DEV)
    M = ops.transparse_premul(Wd, md) if premul else None
    got = {}
    for key, form, split in (("old", 1, False), ("one", 0, False), ("split", 0, True), ("split2", 0, True)):
        st = torch.empty((B, 2), dtype=torch.float32, device=DEV)
        s = ops.transparse_score_raw(mode, ed, rd, Wd, md, pos.to(DEV), neg.to(DEV), gamma, stats=st, M=M,
                                     forms=dict(transparse_form=form), split=split)
        torch.cuda.synchronize()
        got[key] = (s.cpu().numpy(), st.cpu().numpy())
    bad = np.zeros(B, dtype=bool)
    bad[[3, 5]] = True
    old = got["old"][0][:, 0]
    assert np.array_equal(got["split"][0], got["split2"][0], equal_nan=True)  # deterministic
    assert np.array_equal(got["split"][1], got["split2"][1], equal_nan=True)
    for key in ("one", "split"):
        new = got[key][0][:, 0]
        assert np.isnan(new[bad]).all() and np.isnan(old[bad]).all()
        assert np.abs(new[~bad] - old[~bad]).max() <= 1e-5 * max(1.0, np.abs(old[~bad]).max()), key
    new = got["split"][0][:, 0]
    ok_pos = pos.clone()
    ok_pos[3, 1], ok_pos[5, 0] = 0, 0
    ref, _ = _oracle(ent, rel, W, mask, ok_pos, neg, mode, gamma)
    assert rel_close(new[~bad], ref[~bad, 0]) <= 1e-4


@pytest.mark.parametrize("mode,N", [(0, 256), (0, 300), (0, 96), (1, 256)])
@pytest.mark.parametrize("premul", [False, True])
def test_step_forward_fused_is_bitwise_the_two_calls(mode, N, premul):
    """kge_transparse_step_forward (both calls of supervisor.py:17-18 and their reductions in one entry point:
    the head-batch row reduction in ts_fwd_x3s_kernel's epilogue when one block holds the row, N <= 256; the
    positives' logsigmoid in the split form's finish; the standalone reduction launches otherwise) is bitwise
    transparse_score + neg_reduce + log_sigmoid, NaN rows included; and TFKGEModel.step_forward under no_grad
    takes it."""
    E, R, d, B, gamma = 300, 4, 500, 70, 12.0
    ent, rel, W, mask = _tables(E, R, d, seed=7)
    pos, neg = _batch(E, R, B, N, seed=13)
    pos[4, 1] = R + 1  # out-of-range relation: NaN scores
    ed, rd, Wd, md, pd, nd = ent.to(DEV), rel.to(DEV), W.to(DEV), mask.to(DEV), pos.to(DEV), neg.to(DEV)
    M = ops.transparse_premul(Wd, md) if premul else None
    ns, on, ps, op = ops.transparse_step_forward_raw(mode, ed, rd, Wd, md, pd, nd, gamma, M=M)
    ref_ns = ops.transparse_score_raw(mode, ed, rd, Wd, md, pd, nd, gamma, M=M)
    ref_on = ops.neg_reduce_raw(ref_ns, 1.0, True)
    ref_ps = ops.transparse_score_raw(3, ed, rd, Wd, md, pd, None, gamma, M=M).reshape(-1)
    ref_op = ops.log_sigmoid_raw(ref_ps)
    torch.cuda.synchronize()
    for got, ref in ((ns, ref_ns), (on, ref_on), (ps, ref_ps), (op, ref_op)):
        assert torch.equal(torch.nan_to_num(got, nan=7.0), torch.nan_to_num(ref.reshape(got.shape), nan=7.0))
    assert torch.isnan(on[4]) and not torch.isnan(on[:4]).any()
    m = TFKGEModel("TranSparse", E, R, d, gamma, device=DEV, seed=3)
    with torch.no_grad():
        n1, p1 = m.step_forward(pd, nd, mode)
    n2, p2 = m(((pd, nd), mode)), m(((pd, nd), 3))
    assert torch.equal(torch.nan_to_num(n1, nan=7.0), torch.nan_to_num(n2.detach(), nan=7.0))
    assert torch.equal(torch.nan_to_num(p1, nan=7.0), torch.nan_to_num(p2.detach(), nan=7.0))
