"""bench.shard_sim_bench alone (the simulated 8-rank C4 step on one GPU): rank 0's forward and train-step
kernels. python scripts/shard_sim.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    import customknowledgegraphembedding_amd as kge
    from customknowledgegraphembedding_amd import ops
    from customknowledgegraphembedding_amd._lib import FN_IDS
    bench.kge, bench.ops, bench.FN_IDS = kge, ops, FN_IDS
    out = bench.shard_sim_bench(torch.device("cuda:0"))
    print(json.dumps({k: out[k] for k in ("rank_step_kernels_us", "rank_train_step_kernels_us")}), flush=True)


if __name__ == "__main__":
    main()
