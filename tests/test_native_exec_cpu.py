"""CPU tests of the native row-sharded executor's boundary (kge_comm_*, kge_shard_exec_*; include/kge_hip.h):
sizes and argument checks that return before any HIP or RCCL call. The executor's results are checked on
the GPU (tests/test_native_exec_gpu.py, tests/test_rccl_gpu.py)."""
import ctypes

import pytest
import torch

import customknowledgegraphembedding_amd as kge
from customknowledgegraphembedding_amd.distributed import ShardedKGE

EINVAL = -22


def _lib():
    return kge.load()


def test_workspace_size_bounds_every_buffer():
    lib = _lib()
    Bg, N, d, W, K = 4096, 1024, 500, 8, 2
    n = lib.kge_shard_exec_workspace_size(Bg, N, d, W, K)
    # three plan slots (each with its [Bg, N+1] bucket of int2) + W copies of the query rows + the score buffers
    slot = Bg * (N + 1) * 8 + 2 * W * Bg * 4
    assert n >= 3 * slot + W * Bg * d * 4 + Bg * d * 4 + Bg * (N + 1) * 4
    assert n < 3 * slot + 2 * (W * Bg * d * 4 + Bg * d * 4 + Bg * (N + 1) * 4)
    assert lib.kge_shard_exec_workspace_size(Bg, N, d, W, 3) == EINVAL  # chunks must divide the world
    assert lib.kge_shard_exec_workspace_size(Bg + 1, N, d, W, K) == EINVAL  # the batch must split over ranks
    assert lib.kge_shard_exec_workspace_size(Bg, N, d, 65, 1) == EINVAL
    assert lib.kge_shard_exec_host_ints(8, 2) == 3 * (64 + 16)
    assert lib.kge_shard_exec_host_ints(0, 1) == EINVAL


def test_create_rejects_bad_arguments_before_any_hip_call():
    lib = _lib()
    h = ctypes.c_void_p()
    ws = ctypes.c_void_p(1 << 20)  # never dereferenced: every call below fails its checks first
    host = ctypes.c_void_p(1 << 20)
    Bg, N, d, W, K = 64, 40, 16, 8, 2
    need = lib.kge_shard_exec_workspace_size(Bg, N, d, W, K)
    hi = lib.kge_shard_exec_host_ints(W, K)

    def create(comm=None, flags=0, world=W, rank=0, chunks=K, nbytes=need, hints=hi, wsp=ws):
        return lib.kge_shard_exec_create(ctypes.addressof(h), comm, flags, 1, 1000, 125, d, d, Bg, N, world, rank,
                                         chunks, wsp, nbytes, host, hints)

    assert create() == EINVAL and b"communicator" in lib.kge_last_error()  # W > 1 without comm or probe
    assert create(flags=1, nbytes=need - 1) == EINVAL and b"workspace" in lib.kge_last_error()
    assert create(flags=1, hints=hi - 1) == EINVAL and b"host buffer" in lib.kge_last_error()
    assert create(flags=1, rank=W) == EINVAL
    assert create(flags=1, wsp=ctypes.c_void_p((1 << 20) + 16)) == EINVAL and b"aligned" in lib.kge_last_error()
    assert h.value is None
    assert lib.kge_shard_exec_create(None, None, 0, 1, 1000, 125, d, d, Bg, N, W, 0, K, ws, need, host, hi) == EINVAL


def test_comm_and_loopback_argument_checks():
    lib = _lib()
    h = ctypes.c_void_p()
    idb = ctypes.create_string_buffer(128)
    assert lib.kge_comm_init(ctypes.addressof(h), ctypes.addressof(idb), 0, 0) == EINVAL
    assert lib.kge_comm_init(ctypes.addressof(h), ctypes.addressof(idb), 2, 2) == EINVAL
    assert lib.kge_comm_init(None, ctypes.addressof(idb), 2, 0) == EINVAL
    assert lib.kge_comm_loopback_group(0) is None
    assert lib.kge_comm_loopback_group(65) is None
    assert lib.kge_comm_destroy(None) == 0
    assert lib.kge_shard_exec_destroy(None) == 0
    assert lib.kge_shard_exec_host_wait_us(None, 0) == -1.0
    assert lib.kge_comm_all_to_allv(None, None, None, None, None, None) == EINVAL
    assert lib.kge_shard_exec_plan(None, None, None, 0, 0, None) == EINVAL


def test_sharded_model_needs_a_communicator_for_the_native_step():
    tables = (torch.zeros(100, 8), torch.zeros(3, 8), 12.0, 1.75, 0.0)
    sk = ShardedKGE("DistMult", 100, 3, 8, 12.0, device="cpu", world=4, rank=1, full_tables=tables)
    with pytest.raises(ValueError, match="NativeComm"):
        sk.use_native()
    assert sk.use_native(probe=True) is sk
    sk1 = ShardedKGE("DistMult", 100, 3, 8, 12.0, device="cpu", world=1, rank=0, full_tables=tables)
    assert sk1.use_native() is sk1
