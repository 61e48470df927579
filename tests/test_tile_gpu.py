"""kge_step_forward's row-group x XCD-slice tile form (step_fwd_tile_kernel, forms step_order=tile, the default
for N >= 128): every candidate and positive goes through the same cand_score as the batch-row-major form
(step_fwd_kernel) and the XCD-sliced form (step_fwd_xcd_kernel), so all four outputs must be BITWISE equal
across the three orders, for every score function, both negative modes, any rows-per-block cap, ragged
batches, out-of-range ids, skewed id distributions and the full C2 size (reference: model.py:114-205,
supervisor.py:17-18). The fp64 oracle check of the default (tile) order is in test_configs_gpu.py."""
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd import ops
from customknowledgegraphembedding_amd._lib import FN_IDS

pytestmark = pytest.mark.gpu
DEV = "cuda"
FNS = ["TransE", "DistMult", "ComplEx", "RotatE", "pRotatE", "InterHT"]


def _model(name, E, R, d, seed=0):
    return kge.TFKGEModel(name, E, R, d, 12.0, double_entity_embedding=name in ("ComplEx", "RotatE", "InterHT"),
                          double_relation_embedding=name == "ComplEx", triple_relation_embedding=name == "InterHT",
                          device=DEV, seed=seed)


def _run(m, mode, pos, neg, order, rows=None, q2slots=None):
    """kge_step_forward_ex with an explicit form (kge_forms: the order, the tile kernel's row cap and InterHT
    relation slots)."""
    out = ops.step_forward_raw(FN_IDS[m.model_name], mode, m.entity_embedding.detach(),
                               m.relation_embedding.detach(), m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f,
                               modulus=float(m.modulus.detach().reshape(-1)[0]) if m.model_name == "pRotatE" else 0.0,
                               forms=dict(step_order=order, tile_rows=rows, tile_q2slots=q2slots))
    torch.cuda.synchronize()
    return out


def _same(a, b):
    """Bitwise equal, NaN where the other is NaN (a zero query row gives NaN: no epsilon, Q7)."""
    return all(bool(((x == y) | (torch.isnan(x) & torch.isnan(y))).all()) for x, y in zip(a, b))


def test_order_query_reports_tile_for_large_n():
    lib = kge.load()
    assert lib.kge_step_forward_order(40943, 256) == 2
    assert lib.kge_step_forward_order(40943, 64) == 0


@pytest.mark.parametrize("name", FNS)
@pytest.mark.parametrize("mode", [0, 1])
def test_tile_bitwise_equals_row_and_xcd(name, mode):
    E, R, d, B, N = 3001, 7, 96, 37, 200  # B not a multiple of the rows per block
    m = _model(name, E, R, d)
    g = torch.Generator().manual_seed(5)
    pos = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                       torch.randint(0, E, (B,), generator=g)], 1)
    neg = torch.randint(0, E, (B, N), generator=g)
    # out-of-range ids (zero row, TF-GPU gather), in candidates, positives' tails and query rows
    neg[0, :5] = torch.tensor([-1, E, E + 7, -100, 0])
    pos[1, 2] = E + 3
    pos[2, 0] = -2
    pos[3, 1] = R + 1
    pos, neg = pos.to(DEV), neg.to(DEV)
    want = _run(m, mode, pos, neg, "row")
    assert _same(_run(m, mode, pos, neg, "xcd"), want)
    for rows in (None, 1, 3, 16):
        assert _same(_run(m, mode, pos, neg, "tile", rows), want), rows


@pytest.mark.parametrize("name", FNS)
@pytest.mark.parametrize("mode", [0, 1])
def test_score_indexed_tile_bitwise(name, mode):
    """kge_score_indexed (model(((pos, neg), mode)), model.py:114-205) in the tile order (no positives) equals the
    batch-row-major scorer bitwise, out-of-range ids included."""
    E, R, d, B, N = 2999, 6, 64, 35, 150
    m = _model(name, E, R, d, seed=2)
    g = torch.Generator().manual_seed(13)
    pos = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                       torch.randint(0, E, (B,), generator=g)], 1)
    neg = torch.randint(0, E, (B, N), generator=g)
    neg[2, :3] = torch.tensor([-5, E, E + 1])
    pos, neg = pos.to(DEV), neg.to(DEV)
    mod = float(m.modulus.detach().reshape(-1)[0]) if name == "pRotatE" else 0.0
    outs = []
    for order in ("row", "tile", "xcd"):
        outs.append(ops.score_indexed_raw(FN_IDS[name], mode, m.entity_embedding.detach(),
                                          m.relation_embedding.detach(), m._rel_off, pos, neg, m._D, m._gamma_f,
                                          m._range_f, mod, forms=dict(step_order=order)))
        torch.cuda.synchronize()
    assert _same([outs[1]], [outs[0]]) and _same([outs[2]], [outs[0]])


@pytest.mark.parametrize("mode", [0, 1])
def test_tile_skewed_ids_one_slice_and_tiny_shapes(mode):
    """Every candidate in slice 0 (one block of each row group holds all R (N + 1) items), duplicates of
    one id, N = 1 and B = 1."""
    name, E, R, d = "InterHT", 4000, 5, 64
    m = _model(name, E, R, d, seed=1)
    g = torch.Generator().manual_seed(9)
    for B, N, hi in ((33, 300, 400), (5, 128, 1), (1, 1, E), (17, 1, E)):
        pos = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                           torch.randint(0, hi, (B,), generator=g)], 1).to(DEV)
        neg = torch.randint(0, hi, (B, N), generator=g).to(DEV)
        want = _run(m, mode, pos, neg, "row")
        assert _same(_run(m, mode, pos, neg, "tile"), want), (B, N, hi)


@pytest.mark.parametrize("mode", [0, 1])
def test_tile_interht_relation_slots(mode):
    """InterHT's relation thirds: rows sorted by relation (B <= 2048) with the first runs' thirds in LDS slots and
    the rest read per candidate; many relations (slot overflow), no slots at all, out-of-range relations, and a
    batch too large for the in-block sort (B > 2048, rows in batch order)."""
    g = torch.Generator().manual_seed(11)
    for E, R, B, N, slots in ((2500, 300, 40, 140, None), (2500, 5, 40, 140, 0), (2500, 7, 1500, 128, None),
                              (2500, 3, 2100, 130, None)):
        m = _model("InterHT", E, R, 32)
        pos = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(-1, R + 1, (B,), generator=g),
                           torch.randint(0, E, (B,), generator=g)], 1).to(DEV)
        neg = torch.randint(0, E, (B, N), generator=g).to(DEV)
        want = _run(m, mode, pos, neg, "row")
        assert _same(_run(m, mode, pos, neg, "tile", q2slots=slots), want), (R, B, slots)


@pytest.mark.parametrize("mode", [0, 1])
def test_tile_c2_full_size_bitwise(mode):
    """C2: WN18RR InterHT d=1000 -de -tr, B=512, N=256: tile == XCD-sliced == row-major, bitwise."""
    name, E, R, d, B, N = "InterHT", 40943, 11, 1000, 512, 256
    m = kge.TFKGEModel(name, E, R, d, 24.0, double_entity_embedding=True, triple_relation_embedding=True,
                       device=DEV, seed=0)
    g = torch.Generator().manual_seed(3)
    pos = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                       torch.randint(0, E, (B,), generator=g)], 1).to(DEV)
    neg = torch.randint(0, E, (B, N), generator=g).to(DEV)
    want = _run(m, mode, pos, neg, "xcd")
    assert _same(_run(m, mode, pos, neg, "tile"), want)
    assert _same(_run(m, mode, pos, neg, "row"), want)


@pytest.mark.parametrize("mode", [0, 1])
def test_tile_step_forward_graph_capture_replays_bitwise(mode):
    """The boundary's contract (stream-async, no host sync, graph-capturable): kge_step_forward in the tile
    form and kge_score_indexed captured into a HIP graph replay to the eager outputs bitwise."""
    name, E, R, d, B, N = "InterHT", 3000, 7, 64, 40, 200
    m = _model(name, E, R, d, seed=4)
    g = torch.Generator().manual_seed(21)
    pos = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                       torch.randint(0, E, (B,), generator=g)], 1).to(DEV)
    neg = torch.randint(0, E, (B, N), generator=g).to(DEV)
    ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()

    def call():
        fwd = ops.step_forward_raw(FN_IDS[name], mode, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f)
        sc = ops.score_indexed_raw(FN_IDS[name], mode, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f)
        return list(fwd) + [sc]

    assert kge.load().kge_step_forward_order(E, N) == 2  # the tile form, the default at N >= 128
    want = call()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        call()  # warm-up on a side stream before capture, as torch.cuda.graph expects
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        got = call()
    graph.replay()
    torch.cuda.synchronize()
    assert _same(got, want)
