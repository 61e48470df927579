"""Round 5: the unplanned C2 / C3 / C4 step under tile forms (rows per group, waves per block), same process:
device us per step (events around 40 alternating-mode steps after 10 warm-up, 2 rounds interleaved)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from customknowledgegraphembedding_amd import ops  # noqa: E402
from customknowledgegraphembedding_amd._lib import FN_IDS  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
w = bench.WORKLOADS[wl]
m, batches = bench.make_inputs(w, 0, "cuda")
fn = FN_IDS[w["fn"]]
ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
variants = {"default": None, "rows12": dict(tile_rows=12), "rows8": dict(tile_rows=8), "w16": dict(tile_waves=16),
            "w8": dict(tile_waves=8)}
res = {k: [] for k in variants}
for rnd in range(2):
    for name, fm in variants.items():
        def step(i):
            pos, neg = batches[i % len(batches)]
            return ops.step_forward_raw(fn, i % 2, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f,
                                        forms=fm)
        for i in range(10):
            step(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(40):
            step(i)
        e1.record()
        torch.cuda.synchronize()
        res[name].append(round(e0.elapsed_time(e1) / 40 * 1e3, 1))
print(json.dumps({"workload": wl, **res}))
