"""Round 6: the planned tile step with its sweep direction alternating step by step (kge_step_planner_set_sweep 1:
a step starts on the entity rows the previous step touched last, which the Infinity Cache still holds when the
table exceeds it) against always ascending (0). Device us per step, events around 60 steps after 20 warmup,
rounds interleaved, same batches as bench.py; outputs compared bitwise. Usage: python scripts/sweep_probe.py [wl..]"""
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
dev = torch.device("cuda", 0)


def timed(f, n=60, warm=20):
    for i in range(warm):
        f(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(warm, warm + n):
        f(i)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 2)


for wl in (sys.argv[1:] or ["c2", "c3", "c4"]):
    w = bench.WORKLOADS[wl]
    m, batches = bench.make_inputs(w, 0, dev)
    fn = FN_IDS[w["fn"]]
    res = {"workload": w["name"], "ascending": [], "alternating": []}
    outs = {}
    for rnd in range(3):
        for key, alt in (("ascending", 0), ("alternating", 1)):
            r = bench.StepRunner(m, batches, fn, planned=True)
            r.planner.set_sweep(alt)
            res[key].append(timed(r))
            got = [r(1000 + k) for k in range(2)]  # steps of both directions when alternating
            torch.cuda.synchronize()
            outs[key] = [[t.clone() for t in o] for o in got]
    eq = all(torch.equal(torch.nan_to_num(x), torch.nan_to_num(y))
             for a, b in zip(outs["ascending"], outs["alternating"]) for x, y in zip(a, b))
    res["bitwise_equal"] = eq
    print(json.dumps(res), flush=True)
    del m, batches
    torch.cuda.empty_cache()
