"""Runs bench.shard_sim_bench (one rank of a simulated 8-way row split at the full C4 size) and prints
its JSON; a target for rocprofv3 (python3 scripts/shard_sim.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import customknowledgegraphembedding_amd as kge  # noqa: E402
from customknowledgegraphembedding_amd import ops  # noqa: E402
from customknowledgegraphembedding_amd._lib import FN_IDS  # noqa: E402

bench.kge, bench.ops, bench.FN_IDS = kge, ops, FN_IDS
print(json.dumps(bench.shard_sim_bench(torch.device("cuda", 0))))
