"""Host cost of one rank's row-sharded forward step at W = 8 (bench.rank_host_cost), plus a cProfile
breakdown of where that host time goes. Usage: python scripts/shard_host_probe.py [world] [steps]"""
import cProfile
import json
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import customknowledgegraphembedding_amd  # noqa: F401
    from customknowledgegraphembedding_amd import ops
    from customknowledgegraphembedding_amd._lib import FN_IDS
    from customknowledgegraphembedding_amd.model import TFKGEModel
    bench.ops, bench.FN_IDS, bench.kge = ops, FN_IDS, customknowledgegraphembedding_amd
    device = torch.device("cuda", 0)
    w = bench.WORKLOADS["c4s"]
    full = TFKGEModel("DistMult", w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"], device=device, seed=0)
    tables = (full.entity_embedding.detach(), full.relation_embedding.detach(), full._gamma_f, full._range_f, 0.0)
    out = bench.rank_host_cost(tables, world, device, steps)
    print(json.dumps(out), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    bench.rank_host_cost(tables, world, device, steps)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    # host cost of one RCCL all-to-all through TorchComm (world 1: one piece, this rank to itself), issued
    # async with the device held, as step_forward issues them: the per-call overhead an RCCL step adds
    import socket
    import time
    import torch.distributed as dist
    from customknowledgegraphembedding_amd.distributed import TorchComm
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0, device_id=device)
    c = TorchComm()
    x = torch.zeros(900_000, device=device)
    y = torch.empty_like(x)
    for _ in range(5):
        c.all_to_all(y, x, [x.numel()], [x.numel()], async_op=True).wait()
    torch.cuda.synchronize()
    n = 50
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    hs = [c.all_to_all(y, x, [x.numel()], [x.numel()], async_op=True) for _ in range(n)]
    t1 = time.perf_counter()
    for h in hs:
        h.wait()
    t2 = time.perf_counter()
    ev = torch.cuda.Event()
    ev.record()
    held = not ev.query()
    torch.cuda.synchronize()
    print(json.dumps({"rccl_all_to_all_host_us_per_call": (t1 - t0) / n * 1e6,
                      "rccl_wait_host_us_per_call": (t2 - t1) / n * 1e6, "device_held": held}), flush=True)
    # the same all-to-all through the native communicator (kge_comm_all_to_allv: ncclAllToAllv from C++)
    from customknowledgegraphembedding_amd.distributed import NativeComm
    nc = NativeComm(device=device)
    for _ in range(5):
        nc.all_to_all(y, x, [x.numel()], [x.numel()])
    torch.cuda.synchronize()
    lib = customknowledgegraphembedding_amd.load()
    import ctypes
    sc = (ctypes.c_int64 * 1)(x.numel())
    st = torch.cuda.current_stream().cuda_stream
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    for _ in range(n):
        lib.kge_comm_all_to_allv(nc.handle, x.data_ptr(), ctypes.addressof(sc), y.data_ptr(), ctypes.addressof(sc), st)
    t1 = time.perf_counter()
    ev = torch.cuda.Event()
    ev.record()
    held = not ev.query()
    torch.cuda.synchronize()
    print(json.dumps({"native_rccl_all_to_allv_host_us_per_call": (t1 - t0) / n * 1e6, "device_held": held,
                      "what": "ncclAllToAllv at world 1 (one piece) issued by kge_comm_all_to_allv from a ctypes "
                              "call, device held behind a sleep kernel"}), flush=True)
    nc.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
