"""MI355X-native knowledge-graph-embedding scoring path (drop-in for the hot path of
NguyenThaiHoc1/CustomKnowledgeGraphEmbedding: tensorflow_codes/model.py score plugins,
supervisor.py's negative-sample scoring step, and the upstream KGEModel lookup/score path).

Scoring runs in hand-written gfx950 HIP kernels inside libkge_hip.so (C-ABI: include/kge_hip.h),
called through ctypes on torch's current stream. There is no CPU / eager fallback.
"""
from ._lib import FN_IDS, HEAD_BATCH, SINGLE, TAIL_BATCH, KGEHipError, build_id, load  # noqa: F401
from .model import KGEModel, TFKGEModel  # noqa: F401
from . import ops  # noqa: F401

__all__ = ["TFKGEModel", "KGEModel", "ops", "load", "build_id", "KGEHipError", "FN_IDS",
           "HEAD_BATCH", "TAIL_BATCH", "SINGLE"]
