"""Lower bounds for the fused train forward in the sliced order, on one box.

The fused train forward (`step_fwd_grad_kernel`) runs in batch-row order. A sliced (XCD or tile) order
would gather the same candidate rows with more L2 reuse, but would have to write each (row, slice)'s online-softmax
partial state and merge it (tools/partial_merge_probe.hip times that traffic). This script times, at C2:
  fwd_row / fwd_xcd / fwd_tile — the plain scoring forward (`kge_step_forward`) in each candidate order
                                 (KGE_STEP_ORDER), i.e. what each order's gathers cost without the gradient sums;
  train                        — the train step as shipped (its `step_fwd_grad_kernel` in the kernel trace);
  train_m<K>                   — the same train step with every negative id folded onto K entities (K = 2 048:
                                 16 MB of rows, L2 / Infinity-Cache served; 16 384: 128 MB, Infinity-Cache
                                 served): the fused forward with its gathers cheaper than any order makes them,
                                 i.e. its issue / VALU floor. (K = 64 measures the event counters' atomic
                                 contention instead: ~2 000 events per entity.)
A sliced grad forward costs at least max(sliced plain forward, its VALU floor) + the partial traffic.
Run each variant in its own process under `rocprofv3 --kernel-trace --stats` (the kernel names tell the orders
apart; the train variants share one).
Usage: python3 scripts/train_order_probe.py <variant> [steps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    what = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    import customknowledgegraphembedding_amd as kge
    from customknowledgegraphembedding_amd import ops
    from customknowledgegraphembedding_amd._lib import FN_IDS
    bench.kge, bench.ops, bench.FN_IDS = kge, ops, FN_IDS  # what bench.main binds before its helpers run
    dev = torch.device("cuda:0")
    w = bench.WORKLOADS["c2"]
    m, batches = bench.make_inputs(w, 0, dev)
    if what.startswith("train_m"):  # train_m<K>: negatives folded onto K entities (K x 8 KB rows in the cache)
        k = int(what[7:])
        batches = [(p, n % k) for p, n in batches]
    if what.startswith("fwd_"):
        os.environ["KGE_STEP_ORDER"] = what[4:]

        def step(i):
            p, n = batches[i % len(batches)]
            bench.run_step(m, p, n, i % 2, FN_IDS[w["fn"]])
        for i in range(10):
            step(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(steps):
            step(i)
        e1.record()
        torch.cuda.synchronize()
        out = {"variant": what, "steps": steps, "us_per_step": e0.elapsed_time(e1) * 1e3 / steps}
    else:
        t = bench.train_step_bench(m, batches, steps, 10)
        out = {"variant": what, "steps": steps, "ms_per_step": t["ms_per_step"], "fused": t["fused"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"done in {time.time() - t0:.1f} s", flush=True)
