"""ADVICE r5 (TranSparse workspaces on many relations): device us per kge_transparse_score call with the workspace
the library asks for (split=True) against none (split=False), head-batch (M_r split into bf16 planes per call) and
tail-batch (the column x K split form), on WN18RR's 11 relations and on FB15k-237 / FB15k relation counts, same
process, events around 10 calls, 3 rounds interleaved. Usage: python scripts/ts_many_rel_probe.py"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from customknowledgegraphembedding_amd import _lib, ops  # noqa: E402
from customknowledgegraphembedding_amd.model import TFKGEModel  # noqa: E402

E, d, B, N = 14951, 500, 512, 256
out = {"shape": dict(E=E, d=d, B=B, N=N)}
lib = _lib.load()
for R in (11, 237, 1345):
    m = TFKGEModel("TranSparse", E, R, d, 12.0, device="cuda", seed=0)
    ent, rel, W, mask = m.entity_embedding.detach(), m.relation_embedding.detach(), m.W.detach(), m.mask
    g = np.random.RandomState(1)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)).cuda()
    neg = torch.from_numpy(np.random.RandomState(2).randint(E, size=(B, N))).cuda()
    for mode in (0, 1):
        res = {"workspace_bytes": int(lib.kge_transparse_score_workspace_size(mode, R, B, d)),
               "with_workspace_us": [], "without_us": []}
        outs = {}
        for _ in range(3):
            for key, split in (("with_workspace_us", True), ("without_us", False)):
                for _ in range(2):
                    ops.transparse_score_raw(mode, ent, rel, W, mask, pos, neg, 12.0, split=split)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    s = ops.transparse_score_raw(mode, ent, rel, W, mask, pos, neg, 12.0, split=split)
                e1.record()
                torch.cuda.synchronize()
                res[key].append(round(e0.elapsed_time(e1) / 10 * 1e3, 1))
                outs[key] = s.clone()
        a, b = outs["with_workspace_us"], outs["without_us"]
        res["max_abs_diff"] = float((a - b).abs().max())
        out[f"R{R}_mode{mode}"] = res
        print(json.dumps({f"R{R}_mode{mode}": res}), flush=True)
    del m, ent, rel, W, mask
    ops._WS_CACHE.clear()
    torch.cuda.empty_cache()
print(json.dumps(out))
