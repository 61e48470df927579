"""Round 6: C5's rank call (kge_eval_rank_planes_ex: pair scores, counting plane GEMM, finish) with 256 x 256 (form 1)
and 256 x 192 (form 3) GEMM tiles and LDS-DMA staging (form 4), 4 096 DistMult d=1000 queries x 14 951 entities with a filter, same process,
events around 10 calls, 3 rounds interleaved; ranks compared. Usage: python scripts/rank_form_probe.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import customknowledgegraphembedding_amd as kge  # noqa: E402
from customknowledgegraphembedding_amd import _lib, evaluate  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream().cuda_stream
E, R, d, Bq = 14951, 1345, 1000, 4096
m = kge.KGEModel("DistMult", E, R, d, 24.0, device=dev, seed=0)
g = np.random.RandomState(7)
true = np.stack([g.randint(E, size=200000), g.randint(R, size=200000), g.randint(E, size=200000)], 1)
q = true[:Bq]
ptr, ids = evaluate.build_filter(q, "tail-batch", true)
pos = torch.from_numpy(q).to(dev)
truth = pos[:, 2].contiguous()
fptr, fids = torch.from_numpy(ptr).to(dev), torch.from_numpy(ids).to(dev)
planes = evaluate.entity_planes(m)
want = evaluate.rank_planes(m, pos, "tail-batch", planes, truth, fptr, fids)  # writes the query planes
(qp,) = evaluate._Q_PLANES.values()
(ws,) = evaluate._RANK_WS.values()
res = {"Bq": Bq, "E": E, "d": d, "nfilter": int(len(ids)), "form1_us": [], "form3_us": [], "form4_us": []}
outs = {}
for _ in range(3):
    for form in (1, 3, 4):
        f = _lib.forms(gemm_form=form)
        r = torch.empty(Bq, dtype=torch.int64, device=dev)

        def call():
            assert lib.kge_eval_rank_planes_ex(qp.data_ptr(), Bq, planes.data_ptr(), E, d, Bq, E, truth.data_ptr(),
                                               fptr.data_ptr(), fids.data_ptr(), len(ids), r.data_ptr(), ws.data_ptr(),
                                               ws.numel(), ctypes.addressof(f), st) == 0
        call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            call()
        e1.record()
        torch.cuda.synchronize()
        res[f"form{form}_us"].append(round(e0.elapsed_time(e1) / 10 * 1e3, 1))
        outs[form] = r.clone()
res["ranks_equal"] = all(bool(torch.equal(outs[f], want)) for f in (1, 3, 4))
print(json.dumps(res), flush=True)
