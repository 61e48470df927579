"""Round 6 (DESIGN §7.2's expected 2/4/8-GPU row-sharded step): for W = 2, 4, 8 simulated ranks at the full C4 size
(YAGO3-10 DistMult d=500, N=1024, W x 512 global rows), rank 0's kernels of one forward step (query gather, compact
scoring, finish; device time queued behind a sleep kernel, as bench.shard_sim_bench) and the payload its two
all-to-alls receive per step. The step time at W GPUs is then critical_path + bytes / all-to-all rate (no overlap);
the probe prints it for a range of per-GPU all-to-all rates. Usage: python scripts/shard_scaling_probe.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from customknowledgegraphembedding_amd import ops  # noqa: E402
from customknowledgegraphembedding_amd._lib import FN_IDS  # noqa: E402
from customknowledgegraphembedding_amd.distributed import ShardedKGE, ThreadComm  # noqa: E402
from customknowledgegraphembedding_amd.model import TFKGEModel  # noqa: E402

bench.ops = ops
dev = torch.device("cuda", 0)
w = bench.WORKLOADS["c4s"]
E, d, N, B = w["nentity"], w["hidden_dim"], w["N"], w["B"]
full = TFKGEModel("DistMult", E, w["nrelation"], d, w["gamma"], device=dev, seed=0)
tables = (full.entity_embedding.detach(), full.relation_embedding.detach(), full._gamma_f, full._range_f, 0.0)


def timed(f, n=10):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(50_000_000)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


out = {"workload": w["name"], "per_rank_batch": B, "rates_GBps": [50, 100, 150, 216, 300]}
for world in (1, 2, 4, 8):
    pos, neg, _ = bench._global_batches(w, world, 1, dev)[0]
    if world == 1:
        ent, rel = tables[0], tables[1]
        out["W1_unsharded_step_us"] = timed(lambda: ops.step_forward_raw(FN_IDS["DistMult"], 0, ent, rel, 0, pos, neg, d,
                                                                         full._gamma_f, full._range_f))
        continue
    comm = ThreadComm(world)
    ranks = [ShardedKGE("DistMult", E, w["nrelation"], d, w["gamma"], device=dev, world=world, rank=r, comm=comm,
                        full_tables=tables) for r in range(world)]
    parts = bench.rank0_step_parts(ranks, pos, neg, 0, chunks=1)
    t = {k: timed(parts[k]) for k in ("gather", "score", "finish")}
    cb = ranks[0].collective_bytes(parts["plan"])
    coll = cb["query_rows"] + cb["scores"]
    crit = t["gather"] + t["score"] + t["finish"]
    res = {"kernels_us": t, "critical_path_us": crit, "collective_bytes": cb,
           "step_us_at_rate": {str(r): crit + coll / (r * 1e3) for r in out["rates_GBps"]}}
    res["triples_per_s_at_rate"] = {k: world * B * (N + 1) / (v * 1e-6) for k, v in res["step_us_at_rate"].items()}
    out[f"W{world}"] = res
    print(json.dumps({f"W{world}": res}), flush=True)
    del ranks, comm, parts
    torch.cuda.empty_cache()
print(json.dumps(out))
