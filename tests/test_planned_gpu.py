"""kge_step_forward_planned (ops.StepPlanner): the tile step with its id-only setup (row groups, InterHT's
relation ranking, each group's candidates counting-sorted by XCD slice and entity bucket) made one step ahead
by the previous step's tail blocks, or by kge_step_plan for a run's first batch. The planned step must give
BITWISE the outputs of kge_step_forward on the same batch (itself bitwise across its three forms,
test_tile_gpu.py; against the fp64 oracle in test_configs_gpu.py), for every score function, both modes,
mode changes between consecutive batches, ragged batches, out-of-range ids, skewed ids, InterHT's relation
slots and B > 2 048, and at the full C2 size. Reference: supervisor.py:17-18 (the two calls of one step),
model.py:114-205."""
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd import ops
from customknowledgegraphembedding_amd._lib import FN_IDS

pytestmark = pytest.mark.gpu
DEV = "cuda"
FNS = ["TransE", "DistMult", "ComplEx", "RotatE", "pRotatE", "InterHT"]


def _model(name, E, R, d, seed=0, gamma=12.0):
    return kge.TFKGEModel(name, E, R, d, gamma, double_entity_embedding=name in ("ComplEx", "RotatE", "InterHT"),
                          double_relation_embedding=name == "ComplEx", triple_relation_embedding=name == "InterHT",
                          device=DEV, seed=seed)


def _mod(m):
    return float(m.modulus.detach().reshape(-1)[0]) if m.model_name == "pRotatE" else 0.0


def _batches(E, R, B, N, n, seed, hi=None, rel_lo=0, rel_hi=None):
    g = torch.Generator().manual_seed(seed)
    hi = hi or E
    out = []
    for _ in range(n):
        pos = torch.stack([torch.randint(0, E, (B,), generator=g),
                           torch.randint(rel_lo, rel_hi if rel_hi is not None else R, (B,), generator=g),
                           torch.randint(0, hi, (B,), generator=g)], 1)
        neg = torch.randint(0, hi, (B, N), generator=g)
        out.append((pos.to(DEV), neg.to(DEV)))
    return out


def _unplanned(m, mode, pos, neg):
    return ops.step_forward_raw(FN_IDS[m.model_name], mode, m.entity_embedding.detach(),
                                m.relation_embedding.detach(), m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f,
                                modulus=_mod(m))


def _planner(m, B, N):
    return ops.StepPlanner(FN_IDS[m.model_name], m.entity_embedding.detach(), m.relation_embedding.detach(),
                           m._rel_off, m._D, B, N, m._gamma_f, m._range_f, modulus=_mod(m))


def _same(a, b):
    """Bitwise equal, NaN where the other is NaN (a zero query row gives NaN: no epsilon, Q7)."""
    return all(bool(((x == y) | (torch.isnan(x) & torch.isnan(y))).all()) for x, y in zip(a, b))


def _run_planned(m, batches, modes):
    """plan(batch 0), then step i with batch i + 1 planned in its tail; returns every step's outputs (cloned)."""
    B, N = batches[0][1].shape
    sp = _planner(m, B, N)
    sp.plan(batches[0][0], batches[0][1], modes[0])
    outs = []
    for i in range(len(batches)):
        nxt = (batches[i + 1][0], batches[i + 1][1], modes[i + 1]) if i + 1 < len(batches) else None
        outs.append([t.clone() for t in sp.step(nxt=nxt)])
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("name", FNS)
def test_planned_bitwise_equals_step_forward(name):
    """Four consecutive batches (modes head, tail, tail, head: the plan of each made in the previous step's
    tail), a ragged batch (B not a multiple of the rows per group) and out-of-range ids in candidates,
    positives' tails, query rows and relations."""
    E, R, d, B, N = 3001, 7, 96, 37, 200
    m = _model(name, E, R, d)
    bs = _batches(E, R, B, N, 4, seed=5)
    pos, neg = bs[1]
    neg[0, :5] = torch.tensor([-1, E, E + 7, -100, 0], device=DEV)
    pos[1, 2] = E + 3
    pos[2, 0] = -2
    pos[3, 1] = R + 1
    modes = [0, 1, 1, 0]
    got = _run_planned(m, bs, modes)
    for i, (p, n) in enumerate(bs):
        assert _same(got[i], _unplanned(m, modes[i], p, n)), (name, i)


@pytest.mark.parametrize("mode", [0, 1])
def test_planned_skewed_ids_small_n_and_one_row(mode):
    """Every candidate in slice 0 (one slice holds a group's whole list), duplicates of one id, N below the
    tile form's default threshold (the planned step uses tiles at any N; the unplanned step there is the
    batch-row form, bitwise the same), N = 1 and B = 1."""
    name, E, R, d = "InterHT", 4000, 5, 64
    m = _model(name, E, R, d, seed=1)
    for B, N, hi in ((33, 300, 400), (5, 128, 1), (1, 1, E), (17, 1, E), (20, 64, E)):
        bs = _batches(E, R, B, N, 3, seed=B + N, hi=hi)
        got = _run_planned(m, bs, [mode, 1 - mode, mode])
        for i, (p, n) in enumerate(bs):
            assert _same(got[i], _unplanned(m, [mode, 1 - mode, mode][i], p, n)), (B, N, hi, i)


@pytest.mark.parametrize("mode", [0, 1])
def test_planned_interht_relation_ranks(mode):
    """InterHT's rows ranked by relation in the plan (B <= 2 048) with more relations than LDS slots,
    out-of-range relations, and a batch too large for the ranking (B > 2 048: rows in batch order)."""
    for E, R, B, N in ((2500, 300, 40, 140), (2500, 7, 1500, 128), (2500, 3, 2100, 130)):
        m = _model("InterHT", E, R, 32)
        bs = _batches(E, R, B, N, 2, seed=R, rel_lo=-1, rel_hi=R + 1)
        got = _run_planned(m, bs, [mode, mode])
        for i, (p, n) in enumerate(bs):
            assert _same(got[i], _unplanned(m, mode, p, n)), (R, B, i)


def test_planned_c2_full_size_bitwise():
    """C2: WN18RR-sized InterHT d=1000 -de -tr, B=512, N=256, three batches alternating head / tail."""
    name, E, R, d, B, N = "InterHT", 40943, 11, 1000, 512, 256
    m = kge.TFKGEModel(name, E, R, d, 24.0, double_entity_embedding=True, triple_relation_embedding=True,
                       device=DEV, seed=0)
    bs = _batches(E, R, B, N, 3, seed=3)
    modes = [0, 1, 0]
    got = _run_planned(m, bs, modes)
    for i, (p, n) in enumerate(bs):
        assert _same(got[i], _unplanned(m, modes[i], p, n)), i


def test_planned_plan_is_a_snapshot_of_the_ids():
    """The plan holds the batch's ids: a step reads none of pos / neg, so overwriting them after the plan was
    made does not change that step's outputs."""
    E, R, d, B, N = 2000, 5, 64, 24, 160
    m = _model("RotatE", E, R, d, seed=7)
    (pos, neg), = _batches(E, R, B, N, 1, seed=17)
    want = _unplanned(m, 1, pos, neg)
    sp = _planner(m, B, N)
    p2, n2 = pos.clone(), neg.clone()
    sp.plan(p2, n2, 1)
    p2.random_(0, E)
    n2.random_(0, E)
    got = sp.step()
    torch.cuda.synchronize()
    assert _same(got, want)


def test_planned_wrong_plan_makes_outputs_nan_and_bad_calls_fail():
    """A plan of another batch shape (here: another mode) makes every output NaN instead of silently wrong
    scores; a step whose next plan is the plan it reads, a missing plan, and a shape the tile form cannot take
    are refused."""
    E, R, d, B, N = 2000, 5, 64, 24, 160
    m = _model("DistMult", E, R, d, seed=2)
    (pos, neg), = _batches(E, R, B, N, 1, seed=4)
    lib = kge.load()
    fn = FN_IDS["DistMult"]
    ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
    nbytes = lib.kge_step_plan_size(fn, E, ent.stride(0), R, rel.stride(0), 0, B, N, d)
    assert nbytes > 0
    plan = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    other = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    assert lib.kge_step_plan(fn, 0, E, ent.stride(0), R, rel.stride(0), 0, pos.data_ptr(), neg.data_ptr(),
                             neg.stride(0), B, N, d, plan.data_ptr(), st) == 0
    ns = torch.zeros(B, N, device=DEV)
    on, op, ps = (torch.zeros(B, device=DEV) for _ in range(3))

    def planned(mode, pl, nxt_plan=None):
        return lib.kge_step_forward_planned(fn, mode, ent.data_ptr(), E, ent.stride(0), rel.data_ptr(), R,
                                            rel.stride(0), 0, B, N, d, m._gamma_f, m._range_f, 0.0, 1.0, 1, pl,
                                            pos.data_ptr(), neg.data_ptr(), neg.stride(0), 1, nxt_plan,
                                            ns.data_ptr(), N, on.data_ptr(), ps.data_ptr(), op.data_ptr(), st)
    assert planned(1, plan.data_ptr()) == 0  # the plan was made for head-batch (mode 0)
    torch.cuda.synchronize()
    assert bool(torch.isnan(ns).all()) and bool(torch.isnan(op).all()) and bool(torch.isnan(on).all())
    assert planned(0, plan.data_ptr(), plan.data_ptr()) != 0
    assert planned(0, None) != 0
    assert planned(0, plan.data_ptr(), other.data_ptr()) == 0
    torch.cuda.synchronize()
    want = _unplanned(m, 0, pos, neg)
    assert _same([on, op, ns, ps], want)
    # N + 1 past the 16-bit column of a plan item, or a width past the tile kernel's registers: no plan
    assert lib.kge_step_plan_size(fn, E, ent.stride(0), R, rel.stride(0), 0, B, 70000, d) == 0
    assert lib.kge_step_plan_size(fn, E, 4096, R, 4096, 0, B, N, 4096) == 0
    assert not ops.StepPlanner.available(fn, ent, rel, 0, d, B, 70000)
    with pytest.raises(RuntimeError):
        _planner(m, B, N).step()


def test_planned_plan_of_the_other_row_order_makes_outputs_nan():
    """a plan made for a score function without the relation sort (DistMult) has InterHT's batch shape,
    but not its row order: the InterHT planned step refuses it by the header's sort flag (NaN outputs)."""
    E, R, d, B, N = 2000, 5, 64, 24, 160
    lib = kge.load()
    mi = _model("InterHT", E, R, d, seed=3)
    (pos, neg), = _batches(E, R, B, N, 1, seed=5)
    ent, rel = mi.entity_embedding.detach(), mi.relation_embedding.detach()
    st = torch.cuda.current_stream().cuda_stream
    nb_i = lib.kge_step_plan_size(FN_IDS["InterHT"], E, ent.stride(0), R, rel.stride(0), mi._rel_off, B, N, d)
    nb_d = lib.kge_step_plan_size(FN_IDS["DistMult"], E, d, R, d, 0, B, N, d)
    assert nb_i > 0 and nb_d > 0
    plan = torch.empty(max(nb_i, nb_d), dtype=torch.uint8, device=DEV)
    own = torch.empty(max(nb_i, nb_d), dtype=torch.uint8, device=DEV)
    assert lib.kge_step_plan(FN_IDS["InterHT"], 1, E, ent.stride(0), R, rel.stride(0), mi._rel_off, pos.data_ptr(),
                             neg.data_ptr(), neg.stride(0), B, N, d, own.data_ptr(), st) == 0
    assert lib.kge_step_plan(FN_IDS["DistMult"], 1, E, d, R, d, 0, pos.data_ptr(), neg.data_ptr(), neg.stride(0), B,
                             N, d, plan.data_ptr(), st) == 0
    torch.cuda.synchronize()
    h_own, h_other = own[:28].view(torch.int32).cpu(), plan[:28].view(torch.int32).cpu()
    assert torch.equal(h_own[:6], h_other[:6]) and int(h_own[6]) != int(h_other[6])  # only the sort flag differs
    ns = torch.zeros(B, N, device=DEV)
    on, op, ps = (torch.zeros(B, device=DEV) for _ in range(3))
    assert lib.kge_step_forward_planned(FN_IDS["InterHT"], 1, ent.data_ptr(), E, ent.stride(0), rel.data_ptr(), R,
                                        rel.stride(0), mi._rel_off, B, N, d, mi._gamma_f, mi._range_f, 0.0, 1.0, 1,
                                        plan.data_ptr(), pos.data_ptr(), neg.data_ptr(), neg.stride(0), 1, None,
                                        ns.data_ptr(), N, on.data_ptr(), ps.data_ptr(), op.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert bool(torch.isnan(ns).all()) and bool(torch.isnan(on).all()) and bool(torch.isnan(op).all())


def test_planner_step_checks_caller_outputs():
    """StepPlanner.step(out=...) refuses outputs of the wrong shape, strides, dtype or device."""
    E, R, d, B, N = 2000, 5, 64, 24, 160
    m = _model("DistMult", E, R, d, seed=2)
    (pos, neg), = _batches(E, R, B, N, 1, seed=4)
    sp = _planner(m, B, N)
    sp.plan(pos, neg, 0)
    good = sp.outputs()
    bad = [
        (good[0], good[1], torch.empty(N, B, device=DEV).t(), good[3]),          # transposed strides
        (good[0], good[1], torch.empty(B, N + 1, device=DEV)[:, :N], good[3]),   # padded rows
        (good[0].double(), good[1], good[2], good[3]),                           # dtype
        (good[0], good[1], good[2], torch.empty(B + 1, device=DEV)),             # shape
        (good[0].cpu(), good[1], good[2], good[3]),                              # device
        good[:3],
    ]
    for out in bad:
        with pytest.raises((ValueError, TypeError)):
            sp.step(out=out)
    got = sp.step(out=good)
    torch.cuda.synchronize()
    assert _same(got, _unplanned(m, 0, pos, neg))
