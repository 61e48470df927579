"""Round-5 probe: the C2 step with and without its plan made ahead, and where the plan is made.
Device time per step (events around 50 steps after 20 warmup), same batches as bench.py's C2 line:
  unplanned           kge_step_forward (setup inside the tile kernel)
  planned_tail        kge_step_forward_planned, next plan in the tile launch's tail blocks
  planned_standalone  kge_step_plan as its own launch, then the planned step without a next plan
Usage: python scripts/plan_probe.py [workload]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from customknowledgegraphembedding_amd import ops  # noqa: E402
from customknowledgegraphembedding_amd._lib import FN_IDS  # noqa: E402

bench.ops = ops
wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
w = bench.WORKLOADS[wl]
dev = torch.device("cuda", 0)
m, batches = bench.make_inputs(w, 0, dev)
fn = FN_IDS[w["fn"]]


def timed(f, n=50, warm=20):
    for i in range(warm):
        f(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(warm, warm + n):
        f(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


res = {}
plain = bench.StepRunner(m, batches, fn, planned=False)
res["unplanned"] = timed(plain)
# one mode only (the same kernel object every step) against alternating modes (the default above): what a
# mode switch costs per step
res["unplanned_head_only"] = timed(lambda i: plain(i, 0))
res["unplanned_tail_only"] = timed(lambda i: plain(i, 1))
r = bench.StepRunner(m, batches, fn, planned=True)
res["planned_tail"] = timed(r)
res["planned_tail_head_only"] = timed(lambda i: r(i, 0))
sp = bench.StepRunner(m, batches, fn, planned=True).planner


def standalone(i):
    pos, neg = batches[i % len(batches)]
    sp.plan(pos, neg, i % 2)
    sp.step()


res["planned_standalone"] = timed(standalone)


def plan_only(i):
    pos, neg = batches[i % len(batches)]
    sp.plan(pos, neg, i % 2)


res["plan_kernel_alone"] = timed(plan_only)
res["workload"] = w["name"]
print(json.dumps(res), flush=True)
