"""CPU tests of the C-ABI boundary: libkge_hip.so loads, exports every symbol include/kge_hip.h
declares, and rejects bad arguments with the documented codes before touching the GPU."""
import ctypes
import os
import re

import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd import _lib, ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kge_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kge_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("kge_score_indexed", "kge_score_dense", "kge_neg_reduce", "kge_score_indexed_bwd",
              "kge_last_error", "kge_abi_version"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_every_declared_symbol():
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_abi_version_and_limits():
    lib = kge.load()
    assert lib.kge_abi_version() == 1
    assert lib.kge_max_dim(4) == 2048
    assert lib.kge_max_dim(99) == 0
    assert lib.kge_score_bwd_workspace_size(4, 1, 512, 256, 1000) >= 0


def test_bad_arguments_are_rejected_without_a_launch():
    lib = kge.load()
    dummy = ctypes.c_void_p(16)
    # unknown score function id
    rc = lib.kge_score_indexed(99, 1, dummy, 10, 4, dummy, 2, 4, 0, dummy, dummy, 4, 2, 4, 4,
                               1.0, 1.0, 0.0, dummy, 4, None)
    assert rc == -22 and b"score function" in lib.kge_last_error()
    # bad mode
    rc = lib.kge_score_indexed(0, 7, dummy, 10, 4, dummy, 2, 4, 0, dummy, dummy, 4, 2, 4, 4,
                               1.0, 1.0, 0.0, dummy, 4, None)
    assert rc == -22 and b"mode" in lib.kge_last_error()
    # missing pos / neg
    rc = lib.kge_score_indexed(0, 1, dummy, 10, 4, dummy, 2, 4, 0, None, dummy, 4, 2, 4, 4,
                               1.0, 1.0, 0.0, dummy, 4, None)
    assert rc == -22
    rc = lib.kge_score_indexed(0, 1, dummy, 10, 4, dummy, 2, 4, 0, dummy, None, 4, 2, 4, 4,
                               1.0, 1.0, 0.0, dummy, 4, None)
    assert rc == -22
    # dimension beyond the register-resident limit
    rc = lib.kge_score_indexed(1, 1, dummy, 10, 4096, dummy, 2, 4096, 0, dummy, dummy, 4, 2, 4, 4096,
                               1.0, 1.0, 0.0, dummy, 4, None)
    assert rc == -95 and b"exceeds" in lib.kge_last_error()
    # empty problems are a successful no-op
    assert lib.kge_score_indexed(0, 1, dummy, 10, 4, dummy, 2, 4, 0, dummy, dummy, 4, 0, 4, 4,
                                 1.0, 1.0, 0.0, dummy, 4, None) == 0
    assert lib.kge_neg_reduce(dummy, 0, 4, 4, 1.0, 1, dummy, None) == 0
    assert lib.kge_neg_reduce(dummy, 2, 0, 4, 1.0, 1, dummy, None) == -22


def test_check_raises_with_message():
    lib = kge.load()
    dummy = ctypes.c_void_p(16)
    rc = lib.kge_score_indexed(0, 9, dummy, 10, 4, dummy, 2, 4, 0, dummy, dummy, 4, 2, 4, 4,
                               1.0, 1.0, 0.0, dummy, 4, None)
    with pytest.raises(kge.KGEHipError, match="mode"):
        _lib.check(rc, "kge_score_indexed")


def test_no_cpu_fallback():
    ent = torch.zeros(10, 8)
    rel = torch.zeros(3, 8)
    pos = torch.zeros(2, 3, dtype=torch.int64)
    neg = torch.zeros(2, 4, dtype=torch.int64)
    with pytest.raises(kge.KGEHipError, match="no CPU fallback"):
        ops.score_indexed_raw(0, 1, ent, rel, 0, pos, neg, 8, 1.0, 1.0)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(kge.KGEHipError, match="not found"):
        _lib.load(str(tmp_path / "nope.so"))


def test_mode_codes_q1():
    assert ops.mode_id(0) == kge.HEAD_BATCH
    assert ops.mode_id(1) == kge.TAIL_BATCH
    assert ops.mode_id(2) == kge.TAIL_BATCH  # model.py:124: anything but 0 is tail-batch
    assert ops.mode_id(3) == kge.SINGLE
    assert ops.mode_id("head-batch") == kge.HEAD_BATCH
    assert ops.mode_id(torch.tensor(0)) == kge.HEAD_BATCH
    with pytest.raises(ValueError):
        ops.mode_id("sideways")


def test_library_is_built_from_this_tree():
    """Provenance: kge_source_hash() compiled into the library equals the sha256 of this tree's sources
    (Makefile recipe restated by _lib.source_hash), so the binary the GPU runs is these sources."""
    info = kge.build_id()
    assert info["source_hash"] == _lib.source_hash(), "libkge_hip.so is stale: rebuild with make"
    assert info["build_id"].endswith("src:" + info["source_hash"])


def test_sharded_exchange_rejects_bad_arguments():
    lib = kge.load()
    d = ctypes.c_void_p(16)
    # chunks must divide the world; world limit; modes
    assert lib.kge_shard_plan(d, d, 4, 8, 4, 100, 4, 3, 0, 0, 0, d, d, d, d, d, None, None, None) == -22
    assert lib.kge_shard_plan(d, d, 4, 130, 4, 1000, 65, 1, 0, 0, 0, d, d, d, d, d, None, None, None) == -95
    assert lib.kge_shard_plan(d, d, 4, 8, 4, 100, 2, 1, 3, 0, 0, d, d, d, d, d, None, None, None) == -22
    assert lib.kge_shard_plan(d, d, 4, 9, 4, 100, 2, 1, 1, 0, 0, d, d, d, d, d, None, None, None) == -22  # Bg % W
    assert lib.kge_shard_plan(d, d, 4, 0, 4, 100, 2, 1, 1, 0, 0, d, d, d, d, d, None, None, None) == 0    # empty
    # the bucket: both arrays or neither, the forward's flags and a valid rank
    assert lib.kge_shard_plan(d, d, 4, 8, 4, 100, 2, 1, 1, 0, 0, d, d, d, d, d, d, None, None) == -22
    rc = lib.kge_shard_plan(d, d, 4, 8, 4, 100, 2, 1, 0, 1, 0, d, d, d, d, d, d, d, None)
    assert rc == -22 and b"bucket" in lib.kge_last_error()
    assert lib.kge_shard_plan(d, d, 4, 8, 4, 100, 2, 1, 0, 0, 2, d, d, d, d, d, d, d, None) == -22
    # compact scoring: rows must be whole homes; the negative mode, not single
    rc = lib.kge_shard_score(1, 1, d, 8, 4, d, d, 2, 4, 0, d, 10, 4, 0, d, 3, 4, 4, 1.0, 1.0, 0.0,
                             d, d, d, d, d, 2, 0, 2, 0, d, None)
    assert rc == -22 and b"whole homes" in lib.kge_last_error()
    rc = lib.kge_shard_score(1, 3, d, 8, 4, d, d, 2, 4, 0, d, 10, 4, 0, d, 4, 4, 4, 1.0, 1.0, 0.0,
                             d, d, d, d, d, 2, 0, 2, 0, d, None)
    assert rc == -22 and b"mode" in lib.kge_last_error()
    assert lib.kge_shard_finish(d, d, d, d, d, 4, 8, 4, 100, 2, 2, 0, 1.0, 1, d, 4, d, d, d, None) == -22
    assert lib.kge_shard_gather_queries(d, 10, 4, 0, d, 8, 3, 0, 4, 2, 0, 0, 0, d, d, d, d, d, None) == -22


def test_step_forward_order_choice_reads_no_environment(monkeypatch):
    """kge_step_forward_order (host-only): the tile form (2) for N >= 128, one launch (0) below, and tables past
    the sort keys' range take the one-launch form. The library reads no environment: a form is chosen only
    through the _ex entry points' kge_forms."""
    lib = kge.load()
    for name in ("row", "xcd", "tile"):
        monkeypatch.setenv("KGE_STEP_ORDER", name)  # the old A/B knob: ignored
        assert lib.kge_step_forward_order(40943, 256) == 2    # C2
    assert lib.kge_step_forward_order(123182, 1024) == 2  # C4
    assert lib.kge_step_forward_order(40943, 127) == 0
    assert lib.kge_step_forward_order(8 << 25, 256) == 0


def test_workspace_queries_are_host_arithmetic():
    """The round-5 workspace and plane-size queries (no GPU needed): TranSparse head-batch M_r planes
    [R][3][K / 16][columns rounded to 256][16] bf16, the single / tail-batch partial projections
    [ksplit][B][xsplit 128] fp32, the step's maximum of the two, and the bf16x3 planes of a [rows, K] matrix."""
    lib = _lib.load()
    R, B, d = 11, 512, 500
    planes = R * 3 * ((d + 15) // 16) * ((d + 255) // 256 * 256) * 16 * 2
    ksplit, xsplit = ((d + 15) // 16 + 7) // 8, (d + 127) // 128
    xk = ksplit * B * xsplit * 128 * 4
    assert lib.kge_transparse_score_workspace_size(0, R, B, d) == planes
    assert lib.kge_transparse_score_workspace_size(3, R, B, d) == xk
    assert lib.kge_transparse_score_workspace_size(1, R, B, d) == xk
    assert lib.kge_transparse_step_workspace_size(R, B, d) == max(planes, xk)
    assert lib.kge_transparse_score_workspace_size(0, R, B, 2048) == 0    # past the planes form's d <= 1024
    assert lib.kge_transparse_score_workspace_size(3, R, B, 100) == 0     # one 128-column, one 128-k range
    # many relations (FB15k-237, FB15k) or few rows per relation: no head-batch planes (the staging
    # split), and no planes past 256 MB; the grouped split's partial projections stay (faster at every count)
    for rr in (237, 1345):
        assert lib.kge_transparse_score_workspace_size(0, rr, B, d) == 0
        assert lib.kge_transparse_score_workspace_size(1, rr, B, d) == xk
        assert lib.kge_transparse_step_workspace_size(rr, B, d) == xk
    assert lib.kge_transparse_score_workspace_size(0, 32, 512, d) == 0      # (32 + 1) x 16 rows > 512
    assert lib.kge_transparse_score_workspace_size(0, 31, 512, d) > 0
    assert lib.kge_transparse_score_workspace_size(0, 60, 8192, 1024) == 0  # 60 x 6.3 MB of planes > 256 MB
    assert lib.kge_split_bf16x3_bytes(4096, 1000) == 3 * 4096 * 1008 * 2
    assert lib.kge_split_bf16x3_bytes(7, 36) == 3 * 7 * 48 * 2
