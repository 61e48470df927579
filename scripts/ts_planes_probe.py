"""Round 5: TranSparse head-batch forward at c6, same process: M_r split once per call into bf16 planes
(ts_mplanes_kernel + ts_fwd_x3s_kernel<.., true>, the workspace form) against the in-kernel split
(ts_fwd_x3s_kernel<.., false>, no workspace); device us per call (events around 20 calls, 3 rounds interleaved)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from customknowledgegraphembedding_amd import ops  # noqa: E402
from customknowledgegraphembedding_amd.model import TFKGEModel  # noqa: E402

E, R, d, B, N = 40943, 11, 500, 512, 256
m = TFKGEModel("TranSparse", E, R, d, 12.0, device="cuda", seed=0)
ent, rel, W, mask = m.entity_embedding.detach(), m.relation_embedding.detach(), m.W.detach(), m.mask
g = np.random.RandomState(1)
pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)).cuda()
neg = torch.from_numpy(np.random.RandomState(2).randint(E, size=(B, N))).cuda()
M = ops.transparse_premul(W, mask)
res = {"planes": [], "staging": []}
outs = {}
for rnd in range(3):
    for name, split in (("planes", True), ("staging", False)):
        for _ in range(3):
            ops.transparse_score_raw(0, ent, rel, W, mask, pos, neg, 12.0, M=M, split=split)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            s = ops.transparse_score_raw(0, ent, rel, W, mask, pos, neg, 12.0, M=M, split=split)
        e1.record()
        torch.cuda.synchronize()
        res[name].append(round(e0.elapsed_time(e1) / 20 * 1e3, 1))
        outs[name] = s
res["bitwise_equal"] = bool(torch.equal(torch.nan_to_num(outs["planes"]), torch.nan_to_num(outs["staging"])))
print(json.dumps(res))
