"""Rank 0's kernels of the 8-rank row-sharded forward (C4: YAGO3-10 DistMult d=500, N=1024, global batch
8 x 512) on one GPU, per chunk count: device time of the plan, the query gathers, the compact scoring
(negatives and positives) and the finish, queued behind a sleep kernel so the events bracket GPU work only.
Run it under `rocprofv3 --kernel-trace --stats` to cross-check the per-kernel durations.

    python scripts/shard_probe.py [--chunks 1,2,4] [--reps 20] [--mode 0]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from customknowledgegraphembedding_amd.distributed import ShardedKGE  # noqa: E402
from customknowledgegraphembedding_amd.model import TFKGEModel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--chunks", default="1,2,4")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--mode", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    w = bench.WORKLOADS["c4s"]
    E, d = w["nentity"], w["hidden_dim"]
    pos, neg, _ = bench._global_batches(w, a.world, 1, dev)[0]
    full = TFKGEModel("DistMult", E, w["nrelation"], d, w["gamma"], device=dev, seed=0)
    tables = (full.entity_embedding.detach(), full.relation_embedding.detach(), full._gamma_f, full._range_f, 0.0)
    ranks = [ShardedKGE("DistMult", E, w["nrelation"], d, w["gamma"], device=dev, world=a.world, rank=r,
                        full_tables=tables) for r in range(a.world)]

    def timed(f):
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(50_000_000)
        e0.record()
        for _ in range(a.reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / a.reps * 1e3, 1)

    out = {"order": os.environ.get("KGE_STEP_ORDER", "default"), "mode": a.mode, "world": a.world}
    for k in [int(x) for x in a.chunks.split(",")]:
        p = bench.rank0_step_parts(ranks, pos, neg, a.mode, k)
        r = {name: timed(p[key]) for name, key in (("plan", "plan_fn"), ("gather", "gather"), ("score", "score"),
                                                  ("finish", "finish"))}
        r["total"] = round(r["plan"] + r["gather"] + r["score"] + r["finish"], 1)
        out[f"chunks{p['chunks']}"] = r
        print(json.dumps({f"chunks{p['chunks']}": r}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
