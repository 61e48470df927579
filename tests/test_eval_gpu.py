"""GPU tests of the all-entity evaluation path (upstream test_step): the fp32 MFMA GEMM, exact
filtered ranks vs the oracle's argsort-based restatement, and the metrics."""
import ctypes

import numpy as np
import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd import _lib, evaluate
from oracle import kge_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N,K", [(1, 1, 4), (37, 300, 64), (128, 128, 16), (129, 257, 1000), (1024, 1500, 2000),
                                   (5, 14951, 1000)])
def test_gemm_nt_f32_mfma(M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    Bm = torch.randn(N, K, generator=g, dtype=torch.float64)
    a, b = A.float().to(DEV), Bm.float().to(DEV)
    C = torch.empty(M, N, device=DEV)
    rc = _lib.load().kge_gemm_nt(a.data_ptr(), K, b.data_ptr(), K, C.data_ptr(), N, M, N, K,
                                 torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    ref = a.double().cpu() @ b.double().cpu().T
    scale = (a.double().cpu().abs() @ b.double().cpu().abs().T).clamp_min(1.0)
    assert float(((C.double().cpu() - ref).abs() / scale).max()) < 1e-6


def test_gemm_asymmetric_identity_layout():
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    K = 64
    A = torch.eye(64, K, device=DEV)
    Bm = torch.arange(96 * K, dtype=torch.float32, device=DEV).reshape(96, K) % 97
    C = torch.empty(64, 96, device=DEV)
    assert _lib.load().kge_gemm_nt(A.data_ptr(), K, Bm.data_ptr(), K, C.data_ptr(), 96, 64, 96, K,
                                   torch.cuda.current_stream().cuda_stream) == 0
    assert torch.equal(C, Bm.T.contiguous())  # I . B^T is exact in a k-ordered fma chain


@pytest.mark.parametrize("M,N,K", [(1, 1, 4), (37, 300, 64), (128, 128, 16), (129, 257, 1000), (1024, 1500, 2000),
                                   (5, 14951, 1000), (300, 131, 12), (64, 64, 36)])
def test_gemm_nt_bf16x3_matches_fp32_accuracy(M, N, K):
    """kge_gemm_nt_bf16x3 (fp32 operands split into three bf16 terms in registers, six products on the bf16
    MFMA) is as close to the fp64 product as the fp32 MFMA GEMM: per element |C - C64| <= 4e-7 * sum_k |a b|
    (the fp32 path's bound is ~1.5e-7), and never more than 3x the fp32 path's worst error + 1e-7."""
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g, dtype=torch.float64) * torch.logspace(-2, 2, K, dtype=torch.float64)
    Bm = torch.randn(N, K, generator=g, dtype=torch.float64)
    a, b = A.float().to(DEV), Bm.float().to(DEV)
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    C = torch.empty(M, N, device=DEV)
    assert lib.kge_gemm_nt_bf16x3(a.data_ptr(), K, b.data_ptr(), K, C.data_ptr(), N, M, N, K, st) == 0
    ref = a.double().cpu() @ b.double().cpu().T
    scale = (a.double().cpu().abs() @ b.double().cpu().abs().T).clamp_min(1e-30)
    err_x3 = float(((C.double().cpu() - ref).abs() / scale).max())
    assert err_x3 <= 4e-7, err_x3
    C32 = torch.empty(M, N, device=DEV)
    assert lib.kge_gemm_nt(a.data_ptr(), K, b.data_ptr(), K, C32.data_ptr(), N, M, N, K, st) == 0
    err_32 = float(((C32.double().cpu() - ref).abs() / scale).max())
    assert err_x3 <= 3 * err_32 + 1e-7, (err_x3, err_32)


def test_gemm_bf16x3_asymmetric_identity_layout():
    """A = I with an asymmetric B catches a transposed C write or a swapped k half (guide §3)."""
    K = 48
    A = torch.eye(64, K, device=DEV)
    Bm = torch.arange(200 * K, dtype=torch.float32, device=DEV).reshape(200, K) % 97
    C = torch.empty(64, 200, device=DEV)
    assert _lib.load().kge_gemm_nt_bf16x3(A.data_ptr(), K, Bm.data_ptr(), K, C.data_ptr(), 200, 64, 200, K,
                                          torch.cuda.current_stream().cuda_stream) == 0
    want = torch.zeros(64, 200, device=DEV)
    want[:K] = Bm.T  # row m < K of I . B^T is column m of B^T, exact
    assert torch.equal(C, want)


def test_gemm_bf16x3_rejects_unaligned_k():
    a = torch.zeros(4, 6, device=DEV)
    rc = _lib.load().kge_gemm_nt_bf16x3(a.data_ptr(), 6, a.data_ptr(), 6, a.data_ptr(), 4, 4, 4, 6,
                                        torch.cuda.current_stream().cuda_stream)
    assert rc != 0 and b"multiples of 4" in _lib.load().kge_last_error()


CFG = {"DistMult": (False, False, False), "ComplEx": (True, True, False), "TransE": (False, False, False),
       "RotatE": (True, False, False), "InterHT": (True, False, True), "pRotatE": (False, False, False)}


@pytest.mark.parametrize("name", list(CFG))
def test_filtered_ranks_match_oracle(name):
    de, dr, tr = CFG[name]
    E, R, d, gamma = 211, 5, 16, 6.0
    m = kge.KGEModel(name, E, R, d, gamma, de, dr, device=DEV, seed=4) if name != "InterHT" else \
        kge.TFKGEModel(name, E, R, d, gamma, True, False, True, device=DEV, seed=4)
    g = np.random.RandomState(2)
    true = np.stack([g.randint(E, size=400), g.randint(R, size=400), g.randint(E, size=400)], 1)
    test = true[:29]
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    mod = float(m.modulus.detach().reshape(-1)[0]) if name == "pRotatE" else None
    for mode in ("head-batch", "tail-batch"):
        ptr, ids = evaluate.build_filter(test, mode, true)
        pos = torch.from_numpy(test).to(DEV)
        S = evaluate.score_all(m, pos, mode)
        col = 0 if mode == "head-batch" else 2
        got = evaluate.rank_filtered(S, pos[:, col].contiguous(), torch.from_numpy(ptr).to(DEV),
                                     torch.from_numpy(ids).to(DEV)).cpu()
        want = O.eval_ranks(name, ent, rel, torch.from_numpy(test), mode, true, gamma, m._range_f, mod)
        assert torch.equal(got, want), (name, mode, got, want)


def test_test_step_metrics():
    E, R, d = 150, 4, 8
    m = kge.KGEModel("DistMult", E, R, d, 9.0, device=DEV, seed=1)
    g = np.random.RandomState(0)
    true = np.stack([g.randint(E, size=300), g.randint(R, size=300), g.randint(E, size=300)], 1)
    met = evaluate.test_step(m, true[:40], true, batch_size=16)
    ent = m.entity_embedding.detach().cpu().double()
    rel = m.relation_embedding.detach().cpu().double()
    ranks = np.concatenate([O.eval_ranks("DistMult", ent, rel, torch.from_numpy(true[:40]), md, true, 9.0).numpy()
                            for md in ("head-batch", "tail-batch")])
    want = evaluate.metrics_from_ranks(ranks)
    for k in want:
        assert met[k] == pytest.approx(want[k], rel=1e-12)


def test_test_step_without_entity_planes(monkeypatch):
    """a table whose bf16 planes would pass the plane GEMM's 4 GB limit (forced here by lowering
    evaluate.PLANES_MAX_BYTES) gets no planes, and test_step runs on the staging-split GEMM with the same metrics;
    a device allocation failure takes the same path."""
    E, R, d = 150, 4, 8
    m = kge.KGEModel("DistMult", E, R, d, 9.0, device=DEV, seed=1)
    g = np.random.RandomState(0)
    true = np.stack([g.randint(E, size=300), g.randint(R, size=300), g.randint(E, size=300)], 1)
    assert evaluate.entity_planes(m) is not None
    want = evaluate.test_step(m, true[:40], true, batch_size=16)
    monkeypatch.setattr(evaluate, "PLANES_MAX_BYTES", 16)
    assert evaluate.entity_planes(m) is None
    assert evaluate.test_step(m, true[:40], true, batch_size=16) == want
    monkeypatch.setattr(evaluate, "PLANES_MAX_BYTES", (1 << 32) - 16)

    def oom(*a, **k):
        raise torch.OutOfMemoryError("forced")

    monkeypatch.setattr(evaluate, "split_planes", oom)
    assert evaluate.entity_planes(m) is None
    assert evaluate.test_step(m, true[:40], true, batch_size=16) == want


def test_countries_auc_pr_matches_oracle():
    """Upstream test_step with args.countries on the reference's countries_S1 test triples and regions:
    single-mode scores on the GPU, auc_pr vs sklearn on the fp64 oracle's scores."""
    import os
    import types

    from sklearn.metrics import average_precision_score

    from oracle import kge_oracle as O

    gold = os.path.join(os.path.dirname(__file__), "golden")
    z = np.load(os.path.join(gold, "countries_S1_regions.npz"))
    tr = np.load(os.path.join(gold, "countries_S1_train_ids.npz"))
    E, R = int(tr["nentity"]), int(tr["nrelation"])
    m = kge.KGEModel("TransE", E, R, 50, 1.0, device="cuda", seed=5)
    args = types.SimpleNamespace(countries=True, regions=z["regions"].tolist())
    got = evaluate.test_step(m, z["test"], tr["triples"], args)
    sample, y = [], []
    for h, r, t in z["test"].tolist():
        for reg in args.regions:
            sample.append((h, r, reg))
            y.append(1 if reg == t else 0)
    ent, rel = m.entity_embedding.detach().cpu().double(), m.relation_embedding.detach().cpu().double()
    s = O.score("TransE", ent, rel, torch.tensor(sample), None, "single", 1.0)[:, 0].numpy()
    assert abs(got["auc_pr"] - average_precision_score(np.array(y), s)) < 1e-9


@pytest.mark.parametrize("M,N,K,lda", [(1, 1, 4, 4), (37, 300, 64, 64), (257, 513, 1000, 1000), (300, 131, 12, 16),
                                       (1024, 1500, 2000, 2000), (64, 14951, 1000, 1004)])
def test_gemm_split_once_is_bitwise_the_register_split_kernel(monkeypatch, M, N, K, lda):
    """gemm_nt_x3s_kernel (operands split once at staging into bf16 planes, 256 x 256 tiles) against
    gemm_nt_f32x3_kernel (the same six products per 16-k step, split per fragment in the MFMA loop): C is
    bitwise equal, with partial tiles in M, N and K and a padded leading dimension."""
    g = torch.Generator().manual_seed(M + 3 * N + K)
    A = (torch.randn(M, lda, generator=g) * torch.logspace(-2, 2, lda)).to(DEV)
    Bm = torch.randn(N, K, generator=g).to(DEV)
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    out = []
    for form in (1, 0):  # 1: split per fragment in registers (gemm_nt_f32x3_kernel), 0: split once (x3s)
        C = torch.full((M, N + 3), -7.0, device=DEV)
        f = _lib.forms(gemm_form=form)
        assert lib.kge_gemm_nt_bf16x3_ex(A.data_ptr(), lda, Bm.data_ptr(), K, C.data_ptr(), N + 3, M, N, K,
                                         ctypes.addressof(f), st) == 0
        torch.cuda.synchronize()
        out.append(C.cpu())
    assert torch.equal(out[0], out[1])
    assert bool((out[1][:, N:] == -7.0).all())  # nothing written past N


@pytest.mark.parametrize("M,N,K", [(1, 1, 4), (37, 300, 64), (257, 513, 1000), (300, 131, 12), (64, 14951, 1000),
                                   (129, 77, 36)])
def test_gemm_on_presplit_planes_is_bitwise_the_staging_split(M, N, K):
    """kge_split_bf16x3 + kge_gemm_nt_bf16x3_planes (operands split before the GEMM into three bf16 planes, K padded
    to 16 with zeros; no conversion in the GEMM's loop) against kge_gemm_nt_bf16x3 (split at staging): C bitwise
    equal, partial tiles in M and N, K not a multiple of 16 (the staging form needs K % 4 == 0), a padded leading
    dimension of C; nothing written past N."""
    g = torch.Generator().manual_seed(M + 7 * N + K)
    A = (torch.randn(M, K, generator=g) * torch.logspace(-2, 2, K)).to(DEV)
    Bm = torch.randn(N, K, generator=g).to(DEV)
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    want = torch.full((M, N + 3), -7.0, device=DEV)
    assert lib.kge_gemm_nt_bf16x3(A.data_ptr(), K, Bm.data_ptr(), K, want.data_ptr(), N + 3, M, N, K, st) == 0
    ap, bp = evaluate.split_planes(A), evaluate.split_planes(Bm)
    got = torch.full((M, N + 3), -7.0, device=DEV)
    assert lib.kge_gemm_nt_bf16x3_planes(ap.data_ptr(), M, bp.data_ptr(), N, K, got.data_ptr(), N + 3, M, N, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    assert bool((got[:, N:] == -7.0).all())


def test_score_all_with_entity_planes_is_bitwise_the_per_call_split():
    """evaluate.score_all with the pass's entity planes (evaluate.entity_planes, made once per test_step) gives the
    scores of the call that splits the operands itself, bitwise, for DistMult and ComplEx in both modes."""
    for name, de in (("DistMult", False), ("ComplEx", True)):
        m = kge.KGEModel(name, 900, 7, 96, 12.0, double_entity_embedding=de, double_relation_embedding=de,
                         device=DEV, seed=3)
        g = torch.Generator().manual_seed(1)
        pos = torch.stack([torch.randint(0, 900, (70,), generator=g), torch.randint(0, 7, (70,), generator=g),
                           torch.randint(0, 900, (70,), generator=g)], 1).to(DEV)
        planes = evaluate.entity_planes(m)
        for mode in ("head-batch", "tail-batch"):
            a = evaluate.score_all(m, pos, mode).clone()
            b = evaluate.score_all(m, pos, mode, planes=planes)
            torch.cuda.synchronize()
            assert torch.equal(a, b), (name, mode)


@pytest.mark.parametrize("fn,D,B,mode", [("DistMult", 1000, 300, 0), ("DistMult", 36, 70, 1), ("ComplEx", 500, 130, 1),
                                         ("ComplEx", 24, 9, 0)])
def test_eval_query_planes_is_bitwise_query_then_split(fn, D, B, mode):
    """kge_eval_query_planes (the query rows written straight into the GEMM's bf16 planes, the zero pad of the
    last 16-k chunk included) is bitwise kge_eval_query followed by kge_split_bf16x3, and the plane GEMM on it
    gives the same scores; plane rows beyond B are never read."""
    from customknowledgegraphembedding_amd import _lib as L
    lib = L.load()
    E, R = 400, 7
    torch.manual_seed(3)
    d_ent = 2 * D if fn == "ComplEx" else D
    ent = (torch.rand(E, d_ent, device=DEV) - 0.5)
    rel = (torch.rand(R, d_ent, device=DEV) - 0.5)
    g = np.random.RandomState(5)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)).to(DEV)
    K = d_ent
    st = torch.cuda.current_stream().cuda_stream
    fq = L.FN_IDS[fn]
    Q = torch.empty((B, K), dtype=torch.float32, device=DEV)
    assert lib.kge_eval_query(fq, mode, ent.data_ptr(), E, ent.stride(0), rel.data_ptr(), R, rel.stride(0),
                              pos.data_ptr(), B, D, Q.data_ptr(), K, st) == 0
    nb = int(lib.kge_split_bf16x3_bytes(B + 5, K))
    ref = torch.zeros(nb, dtype=torch.uint8, device=DEV)
    got = torch.full((nb,), 0x7F, dtype=torch.uint8, device=DEV)  # garbage everywhere the kernel does not write
    assert lib.kge_split_bf16x3(Q.data_ptr(), B, K, K, ref.data_ptr(), B + 5, st) == 0
    assert lib.kge_eval_query_planes(fq, mode, ent.data_ptr(), E, ent.stride(0), rel.data_ptr(), R, rel.stride(0),
                                     pos.data_ptr(), B, D, got.data_ptr(), B + 5, st) == 0
    torch.cuda.synchronize()
    kp = (K + 15) // 16 * 16
    r = ref.view(torch.bfloat16).view(3, kp // 16, B + 5, 16)[:, :, :B]
    q = got.view(torch.bfloat16).view(3, kp // 16, B + 5, 16)[:, :, :B]
    assert torch.equal(r.view(torch.int16), q.view(torch.int16))
    ep = evaluate.split_planes(ent)
    S1 = torch.empty((B, E), dtype=torch.float32, device=DEV)
    S2 = torch.empty((B, E), dtype=torch.float32, device=DEV)
    assert lib.kge_gemm_nt_bf16x3_planes(ref.data_ptr(), B + 5, ep.data_ptr(), E, K, S1.data_ptr(), E, B, E, st) == 0
    assert lib.kge_gemm_nt_bf16x3_planes(got.data_ptr(), B + 5, ep.data_ptr(), E, K, S2.data_ptr(), E, B, E, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(S1, S2)


@pytest.mark.parametrize("M,N,K", [(1, 1, 4), (37, 300, 64), (257, 513, 1000), (300, 131, 12), (64, 14951, 1000),
                                   (129, 77, 36), (512, 2048, 2000), (300, 700, 48)])
def test_plane_gemm_b_direct_is_bitwise_the_staged_form(M, N, K):
    """gemm_nt_x3d_kernel (B's fragments straight into registers, A staged 32 k per barrier: kge_forms.gemm_form 2)
    and gemm_nt_x3l_kernel (both staged by LDS-DMA copies, three stages: form 4) against gemm_nt_x3p_kernel (both
    operands staged per 16-k chunk: form 1) on the same planes: C bitwise equal,
    with partial tiles in M and N, odd and even 16-k chunk counts (K 1000: 63 chunks; 2000: 125; 48: 3) and a
    padded leading dimension; nothing written past N."""
    g = torch.Generator().manual_seed(M + 5 * N + K)
    A = (torch.randn(M, K, generator=g) * torch.logspace(-2, 2, K)).to(DEV)
    Bm = torch.randn(N, K, generator=g).to(DEV)
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    ap, bp = evaluate.split_planes(A), evaluate.split_planes(Bm)
    out = []
    for form in (1, 2, 3, 4):  # 3: the staged form with 256 x 192 tiles
        C = torch.full((M, N + 3), -7.0, device=DEV)
        f = _lib.forms(gemm_form=form)
        assert lib.kge_gemm_nt_bf16x3_planes_ex(ap.data_ptr(), M, bp.data_ptr(), N, K, C.data_ptr(), N + 3, M, N,
                                                ctypes.addressof(f), st) == 0
        torch.cuda.synchronize()
        out.append(C.cpu())
    for o in out[1:]:
        assert torch.equal(out[0], o)
        assert bool((o[:, N:] == -7.0).all())


@pytest.mark.parametrize("name,E,d,B", [("DistMult", 900, 96, 70), ("ComplEx", 700, 48, 130), ("DistMult", 14951, 1000, 512),
                                        ("ComplEx", 3000, 500, 300)])
def test_rank_planes_equals_score_matrix_ranks(name, E, d, B):
    """kge_eval_rank_planes (the truth's and the filter entries' scores as MFMA tile diagonals, the plane GEMM counting
    per row, the filter correction) gives rank_filtered(score_all(...))'s ranks exactly, without the [B, E] matrix;
    its pair scores are bitwise the GEMM's elements S[q, truth] and S[q, f]. Both modes, a filter of other true
    triples, out-of-range truths (rank_kernel's -inf truth score), and no filter at all."""
    de = name == "ComplEx"
    m = kge.KGEModel(name, E, 7, d, 12.0, double_entity_embedding=de, double_relation_embedding=de, device=DEV, seed=5)
    g = np.random.RandomState(E + d)
    true = np.stack([g.randint(E, size=4 * B), g.randint(7, size=4 * B), g.randint(E, size=4 * B)], 1)
    # a few hub (h, r) / (r, t) pairs so that some queries have long filter lists
    true[B:B + 200, 0] = true[0, 0]
    true[B:B + 200, 1] = true[0, 1]
    true[B + 200:B + 400, 2] = true[1, 2]
    true[B + 200:B + 400, 1] = true[1, 1]
    q = true[:B]
    planes = evaluate.entity_planes(m)
    lib = _lib.load()
    for mode in ("head-batch", "tail-batch"):
        ptr, ids = evaluate.build_filter(q, mode, true)
        col = 0 if mode == "head-batch" else 2
        pos = torch.from_numpy(q).to(DEV)
        truth = pos[:, col].contiguous().clone()
        truth[3] = -1
        truth[5] = E  # out of range: every finite score counts
        fptr, fids = torch.from_numpy(ptr).to(DEV), torch.from_numpy(ids).to(DEV)
        S = evaluate.score_all(m, pos, mode, planes=planes).clone()
        want = evaluate.rank_filtered(S, truth, fptr, fids)
        got = evaluate.rank_planes(m, pos, mode, planes, truth, fptr, fids)
        torch.cuda.synchronize()
        assert torch.equal(got, want), (name, mode)
        # the pair scores in the workspace: [B] truth scores first, the filter entries' after the counts
        (ws,) = evaluate._RANK_WS.values()  # one device, one stream
        ts = ws[:4 * B].view(torch.float32)
        tcpu = truth.cpu()
        ok = (tcpu >= 0) & (tcpu < E)
        idx = torch.arange(B)
        assert torch.equal(ts.cpu()[ok], S.cpu()[idx[ok], tcpu[ok]])
        off = (B * 8 + 15) // 16 * 16
        nf = len(ids)
        fs = ws[off:off + 4 * nf].view(torch.float32).cpu()
        rows = torch.from_numpy(np.repeat(np.arange(B), np.diff(ptr)))
        assert nf > 10 and torch.equal(fs, S.cpu()[rows, torch.from_numpy(ids)])
        got0 = evaluate.rank_planes(m, pos, mode, planes, truth)
        assert torch.equal(got0, evaluate.rank_filtered(S, truth))
        # the counting GEMM with 256 x 256 tiles staged through registers (kge_forms.gemm_form 1), 256 x 192 tiles
        # (3) and LDS-DMA staging (4): the same ranks
        K = m.entity_embedding.shape[1]
        (qpl,) = evaluate._Q_PLANES.values()  # the batch's query planes, as rank_planes wrote them
        for form in (1, 3, 4):
            f3 = _lib.forms(gemm_form=form)
            r3 = torch.empty(B, dtype=torch.int64, device=DEV)
            assert lib.kge_eval_rank_planes_ex(qpl.data_ptr(), B, planes.data_ptr(), E, K, B, E, truth.data_ptr(),
                                               fptr.data_ptr(), fids.data_ptr(), len(ids), r3.data_ptr(),
                                               ws.data_ptr(), ws.numel(), ctypes.addressof(f3),
                                               torch.cuda.current_stream().cuda_stream) == 0
            torch.cuda.synchronize()
            assert torch.equal(r3, want), (name, mode, form)


def test_test_step_ranks_from_planes_equal_the_score_matrix_path(monkeypatch):
    """test_step on the fused rank path (the two-stream RankPipeline) and with it turned off (score_all +
    rank_filtered): the same metrics."""
    E, R, d = 1200, 6, 64
    for name in ("DistMult", "ComplEx"):
        de = name == "ComplEx"
        m = kge.KGEModel(name, E, R, d, 9.0, double_entity_embedding=de, double_relation_embedding=de, device=DEV,
                         seed=2)
        g = np.random.RandomState(3)
        true = np.stack([g.randint(E, size=3000), g.randint(R, size=3000), g.randint(E, size=3000)], 1)
        a = evaluate.test_step(m, true[:300], true, batch_size=128)
        monkeypatch.setattr(evaluate, "_planes_rank_ok", lambda *args, **kw: False)
        b = evaluate.test_step(m, true[:300], true, batch_size=128)
        monkeypatch.undo()
        assert a == b, name


@pytest.mark.parametrize("name,E,d", [("DistMult", 3000, 200), ("ComplEx", 1500, 96)])
def test_rank_pipeline_equals_rank_planes(name, E, d):
    """evaluate.RankPipeline (batches alternating between two streams, each with its own query planes and workspace,
    kge_eval_rank_planes_phases' three phases in order) gives rank_planes' ranks batch by batch: five batches of
    different sizes and modes, CPU and device inputs, a filter, a one-row batch with an empty filter list; and the
    three phases issued one by one on one stream equal the one-call rank."""
    de = name == "ComplEx"
    m = kge.KGEModel(name, E, 5, d, 12.0, double_entity_embedding=de, double_relation_embedding=de, device=DEV, seed=3)
    g = np.random.RandomState(E)
    true = np.stack([g.randint(E, size=6000), g.randint(5, size=6000), g.randint(E, size=6000)], 1)
    planes = evaluate.entity_planes(m)
    sizes = [700, 256, 1, 513, 700]
    batches, want = [], []
    off = 0
    for i, B in enumerate(sizes):
        q = true[off:off + B]
        off += B
        mode = "head-batch" if i % 2 == 0 else "tail-batch"
        ptr, ids = evaluate.build_filter(q, mode, true)
        col = 0 if mode == "head-batch" else 2
        pos, fptr, fids = torch.from_numpy(q), torch.from_numpy(ptr), torch.from_numpy(ids)
        truth = pos[:, col].contiguous().clone()
        batches.append((pos, mode, truth, fptr, fids, int(ptr[-1])))
        want.append(evaluate.rank_planes(m, pos.to(DEV), mode, planes, truth.to(DEV), fptr.to(DEV), fids.to(DEV)).clone())
    torch.cuda.synchronize()
    pipe = evaluate.RankPipeline(m, planes, max(sizes), max(b[5] for b in batches))
    got = []
    for i, (pos, mode, truth, fptr, fids, nf) in enumerate(batches):
        if i % 2:  # device inputs, complete before the submit
            pos, truth, fptr, fids = pos.to(DEV), truth.to(DEV), fptr.to(DEV), fids.to(DEV)
            torch.cuda.synchronize()
        got.append(pipe.submit(pos, mode, truth, fptr, fids, nf))
    # an explicitly empty filter list (filter_ptr all zero, no ids) ranks as no filter at all
    pos0, mode0, truth0 = batches[1][:3]
    empty = pipe.submit(pos0, mode0, truth0, torch.zeros(pos0.shape[0] + 1, dtype=torch.int64),
                        torch.zeros(0, dtype=torch.int64), 0)
    pipe.flush()
    torch.cuda.synchronize()
    for i in range(len(sizes)):
        assert torch.equal(got[i], want[i]), (name, i)
    nofilter = evaluate.rank_planes(m, pos0.to(DEV), mode0, planes, truth0.to(DEV))
    assert torch.equal(empty, nofilter)
    assert torch.equal(evaluate.rank_filtered(evaluate.score_all(m, pos0.to(DEV), mode0, planes=planes), truth0.to(DEV),
                                              torch.zeros(pos0.shape[0] + 1, dtype=torch.int64, device=DEV),
                                              torch.zeros(0, dtype=torch.int64, device=DEV)), nofilter)
    # phases one by one on one stream
    lib = _lib.load()
    pos, mode, truth, fptr, fids, nf = batches[0]
    pos, truth, fptr, fids = pos.to(DEV), truth.to(DEV), fptr.to(DEV), fids.to(DEV)
    B, K = pos.shape[0], m.entity_embedding.shape[1]
    evaluate.rank_planes(m, pos, mode, planes, truth, fptr, fids)  # writes the batch's query planes
    (qpl,) = evaluate._Q_PLANES.values()
    ws = torch.empty(int(lib.kge_eval_rank_planes_workspace_size(B, nf)), dtype=torch.uint8, device=DEV)
    r = torch.full((B,), -5, dtype=torch.int64, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    for ph in (1, 2, 4):
        assert lib.kge_eval_rank_planes_phases(qpl.data_ptr(), B, planes.data_ptr(), E, K, B, E, truth.data_ptr(),
                                               fptr.data_ptr(), fids.data_ptr(), nf, r.data_ptr(), ws.data_ptr(),
                                               ws.numel(), ph, None, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(r, want[0])
    assert lib.kge_eval_rank_planes_phases(qpl.data_ptr(), B, planes.data_ptr(), E, K, B, E, truth.data_ptr(),
                                           fptr.data_ptr(), fids.data_ptr(), nf, r.data_ptr(), ws.data_ptr(),
                                           ws.numel(), 8, None, st) != 0
