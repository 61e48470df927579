"""Device timeline of the native row-sharded executor at W = 8 (one rank, collectives skipped: KGE_EXEC_PROBE),
C4 full size, two batches planned ahead: run under `rocprofv3 --kernel-trace`, then
`python scripts/native_timeline.py --analyze <dir>` prints the per-step wall time, the kernels' busy time
and the idle gaps between them (where cross-stream event hops or host issue would show).
Usage: python scripts/native_timeline.py [chunks] [steps] [one_stream 0/1]"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def analyze(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f))]
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    # the steady state: from the 10th plan kernel to the last kernel
    plan_starts = [s for s, _, n in ks if "plan_count" in n]
    t0, t1 = plan_starts[10], ks[-1][1]
    win = [(s, e, n) for s, e, n in ks if s >= t0]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    nsteps = sum(1 for _, _, n in win if "shard_finish" in n)
    per = {}
    for s, e, n in win:
        k = n.split("(")[0].replace("void ", "").split("::")[-1][:48]
        per.setdefault(k, []).append((e - s) / 1e3)
    print(json.dumps({"steps": nsteps, "wall_us_per_step": (t1 - t0) / 1e3 / max(1, nsteps),
                      "busy_us_per_step": busy / 1e3 / max(1, nsteps),
                      "kernels_us": {k: sum(v) / len(v) for k, v in per.items()},
                      "kernel_counts": {k: len(v) for k, v in per.items()}}, indent=1))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        return analyze(sys.argv[2])
    chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    one = len(sys.argv) > 3 and sys.argv[3] == "1"
    import torch
    import bench
    import customknowledgegraphembedding_amd as kge
    from customknowledgegraphembedding_amd import ops
    from customknowledgegraphembedding_amd._lib import FN_IDS
    from customknowledgegraphembedding_amd.distributed import ShardedKGE
    from customknowledgegraphembedding_amd.model import TFKGEModel
    bench.ops, bench.FN_IDS, bench.kge = ops, FN_IDS, kge
    dev = torch.device("cuda", 0)
    w = bench.WORKLOADS["c4s"]
    full = TFKGEModel("DistMult", w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"], device=dev, seed=0)
    tables = (full.entity_embedding.detach(), full.relation_embedding.detach(), full._gamma_f, full._range_f, 0.0)
    batches = bench._global_batches(w, 8, 4, dev)
    sk = ShardedKGE("DistMult", w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"], device=dev, world=8, rank=0,
                    comm=bench._PrefilledComm(8, 0), full_tables=tables).use_native(probe=True, one_stream=one)
    for i in range(2):
        sk.plan_native(batches[i][0], batches[i][1], i % 2, chunks=chunks)
    for i in range(steps):
        p, q, _ = batches[i % 4]
        np_, nq, _ = batches[(i + 2) % 4]
        sk.step_forward(p, q, i % 2, chunks=chunks, nxt=(np_, nq, i % 2))
    torch.cuda.synchronize()
    print("native timeline run done", flush=True)


if __name__ == "__main__":
    main()
