"""Round 6: the TranSparse head-batch forward ts_fwd_x3s_kernel with its staging written among the MFMAs
(SCHED, transparse_form 0) against the compiler's order (MFMAs first, then the staging; transparse_form 2), at
FB15k-237's shape (E 14 951, d 500, B 512, N 256) on 237 relations with M = mask * W premultiplied, and on 11
relations with M_r split into planes (workspace; c6's form). (The mask-product variant, measured in session F at
613 against 404 us, keeps the compiler's order.) Same process, events
around 10 calls, 6 rounds interleaved (the order alternating); scores compared bitwise. Usage: python scripts/ts_sched_probe.py"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from customknowledgegraphembedding_amd import ops  # noqa: E402
from customknowledgegraphembedding_amd.model import TFKGEModel  # noqa: E402

E, d, B, N = 14951, 500, 512, 256
flop = 6 * 2.0 * B * N * ((d + 255) // 256 * 256) * ((d + 15) // 16 * 16)
for R, case in ((237, "premul"), (11, "planes")):
    m = TFKGEModel("TranSparse", E, R, d, 12.0, device="cuda", seed=0)
    ent, rel, W, mask = m.entity_embedding.detach(), m.relation_embedding.detach(), m.W.detach(), m.mask
    g = np.random.RandomState(1)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)).cuda()
    neg = torch.from_numpy(np.random.RandomState(2).randint(E, size=(B, N))).cuda()
    M = ops.transparse_premul(W, mask) if case == "premul" else None
    split = case == "planes"
    res = {"R": R, "case": case, "sched_us": [], "compiler_order_us": []}
    outs = {}
    for rnd in range(6):
        for key, form in (("sched_us", 0), ("compiler_order_us", 2))[::1 if rnd % 2 == 0 else -1]:
            def call():
                return ops.transparse_score_raw(0, ent, rel, W, mask, pos, neg, 12.0, M=M, split=split,
                                                forms=dict(transparse_form=form))
            call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                s = call()
            e1.record()
            torch.cuda.synchronize()
            res[key].append(round(e0.elapsed_time(e1) / 10 * 1e3, 1))
            outs[key] = s.clone()
    res["bitwise_equal"] = bool(torch.equal(outs["sched_us"], outs["compiler_order_us"]))
    for key in ("sched_us", "compiler_order_us"):
        res[key.replace("_us", "_frac_bf16_peak_call")] = round(flop / (min(res[key]) * 1e-6) / 2.5e15, 3)
    print(json.dumps(res), flush=True)
    del m, ent, rel, W, mask, M
    ops._WS_CACHE.clear()
    torch.cuda.empty_cache()
