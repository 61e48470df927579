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
