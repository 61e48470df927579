"""Why the row-sharded step's host cost reads higher inside bench.py than in a fresh process (A/B, one box).

bench.py measures rank_host_cost at the end of shard_sim_bench (after the 8-thread ThreadComm step); the standalone
scripts/shard_host_probe.py measures it in a fresh process. Variants (argv[1]):
  fresh      rank_host_cost in a fresh process (the probe's setting);
  after_sim  shard_sim_bench as bench.py runs it (rank_host_cost inside, after the simulated 8-rank step);
  after_gc   the same, with gc.collect() + gc.freeze() right before rank_host_cost (the sim's garbage kept out
             of the measured loop's collections).
Prints the host_us_per_rank_step dict as JSON.
"""
import gc
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    what = sys.argv[1]
    import customknowledgegraphembedding_amd as kge
    from customknowledgegraphembedding_amd import ops
    from customknowledgegraphembedding_amd._lib import FN_IDS
    from customknowledgegraphembedding_amd.model import TFKGEModel
    bench.kge, bench.ops, bench.FN_IDS = kge, ops, FN_IDS
    dev = torch.device("cuda:0")
    if what == "fresh":
        w = bench.WORKLOADS["c4s"]
        full = TFKGEModel("DistMult", w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"], device=dev, seed=0)
        tables = (full.entity_embedding.detach(), full.relation_embedding.detach(), full._gamma_f, full._range_f, 0.0)
        out = bench.rank_host_cost(tables, 8, dev)
    else:
        if what == "after_gc":
            inner = bench.rank_host_cost

            def frozen(*a, **k):
                gc.collect()
                gc.freeze()
                return inner(*a, **k)
            bench.rank_host_cost = frozen
        out = bench.shard_sim_bench(dev)["host_us_per_rank_step"]
    print(json.dumps({"variant": what, "python_total": out["python_path"]["total"],
                      "native_step_us": out["native"]["step_us"], "native_blocked_us": out["native"]["blocked_us_per_step"],
                      "native_wall_us": out["native"]["wall_us_per_step"], "gc_counts": gc.get_count(),
                      "gc_frozen": gc.get_freeze_count()}), flush=True)


if __name__ == "__main__":
    main()
