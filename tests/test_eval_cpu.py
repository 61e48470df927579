"""CPU tests of the evaluation host logic: filter CSR construction and metrics."""
import numpy as np

from customknowledgegraphembedding_amd import evaluate


def test_build_filter_matches_upstream_definition():
    true = [(0, 0, 1), (2, 0, 1), (3, 0, 1), (0, 0, 4), (0, 1, 1)]
    q = np.array([[0, 0, 1]])
    ptr, ids = evaluate.build_filter(q, "head-batch", true)
    assert ptr.tolist() == [0, 2] and ids.tolist() == [2, 3]
    ptr, ids = evaluate.build_filter(q, "tail-batch", true)
    assert ptr.tolist() == [0, 1] and ids.tolist() == [4]


def test_metrics():
    m = evaluate.metrics_from_ranks(np.array([1, 2, 4, 20]))
    assert m["MR"] == 6.75
    assert abs(m["MRR"] - (1 + 0.5 + 0.25 + 0.05) / 4) < 1e-12
    assert m["HITS@1"] == 0.25 and m["HITS@3"] == 0.5 and m["HITS@10"] == 0.75


def _eval_worker(rank, world, port, results):
    """gloo rank: evaluate.test_step with the scoring/ranking kernels swapped for oracle versions
    (TEST INFRASTRUCTURE), so the replica orchestration (strided split + rank all-gather) runs on CPU."""
    import os

    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        results[rank] = _run_test_step_with_oracle()
    finally:
        dist.destroy_process_group()


def _run_test_step_with_oracle():
    import torch

    from customknowledgegraphembedding_amd.model import KGEModel
    from oracle import kge_oracle as O

    E, R = 23, 3
    m = KGEModel("TransE", E, R, 8, 6.0, device="cpu", seed=4)
    g = np.random.RandomState(3)
    true = np.stack([g.randint(E, size=40), g.randint(R, size=40), g.randint(E, size=40)], 1)
    test = true[:9]
    ent, rel = m.entity_embedding.detach().double(), m.relation_embedding.detach().double()

    def score_all(model, pos, mode, out=None, planes=None):
        cand = torch.arange(E, dtype=torch.int64).unsqueeze(0).expand(pos.shape[0], E)
        return O.score("TransE", ent, rel, pos, cand, mode, 6.0)

    def rank_filtered(S, truth, fptr, fids):
        ranks = []
        for i in range(S.shape[0]):
            filt = set(fids[int(fptr[i]):int(fptr[i + 1])].tolist())
            st = S[i, int(truth[i])]
            ranks.append(1 + sum(1 for e in range(E) if e != int(truth[i]) and e not in filt and S[i, e] > st))
        return torch.tensor(ranks, dtype=torch.int64)

    saved = evaluate.score_all, evaluate.rank_filtered
    evaluate.score_all, evaluate.rank_filtered = score_all, rank_filtered
    try:
        return evaluate.test_step(m, test, true, batch_size=4)
    finally:
        evaluate.score_all, evaluate.rank_filtered = saved


def test_test_step_replicas_world2_gloo():
    """Multi-replica test_step (each rank ranks a strided share, ranks all-gathered) gives the
    single-process metrics on every rank."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    single = _run_test_step_with_oracle()
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_eval_worker, args=(2, port, results), nprocs=2, join=True)
    for r in range(2):
        for k, v in single.items():
            assert abs(results[r][k] - v) < 1e-12, (k, results[r][k], v)


def test_average_precision_matches_sklearn():
    """evaluate.average_precision == sklearn.metrics.average_precision_score (upstream's auc_pr),
    including tied scores."""
    from sklearn.metrics import average_precision_score

    g = np.random.RandomState(0)
    for n, ties in ((10, False), (200, False), (200, True), (5, True)):
        y = g.randint(2, size=n)
        y[0] = 1
        s = g.rand(n)
        if ties:
            s = np.round(s * 4) / 4
        assert abs(evaluate.average_precision(y, s) - average_precision_score(y, s)) < 1e-12


def test_read_regions(tmp_path):
    """Upstream run.py reads data/countries_S*/regions.list (one entity name per line) into ids."""
    (tmp_path / "regions.list").write_text("oceania\nasia\neurope\n")
    assert evaluate.read_regions(str(tmp_path), {"asia": 7, "europe": 3, "oceania": 9}) == [9, 7, 3]
