"""Does the TranSparse forward's time depend on how the batch rows' relations are spread? The c6 shape
(E=40943, d=500, B=512, N=256, R=11) with (a) random relations (the bench), (b) relations sorted by batch
row, (c) one relation for every row. Same kernel, same bytes; only M_r's reuse in L2 changes."""
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
pos = np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)
neg = torch.from_numpy(np.random.RandomState(2).randint(E, size=(B, N))).cuda()
M = ops.transparse_premul(W, mask)
for name, rr in (("random", pos[:, 1]), ("sorted", np.sort(pos[:, 1])), ("single", np.zeros(B, np.int64))):
    p = pos.copy()
    p[:, 1] = rr
    pt = torch.from_numpy(p).cuda()
    for _ in range(3):
        ops.transparse_score_raw(0, ent, rel, W, mask, pt, neg, 12.0, M=M)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        ops.transparse_score_raw(0, ent, rel, W, mask, pt, neg, 12.0, M=M)
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:8s} {e0.elapsed_time(e1) / 10 * 1e3:8.1f} us", flush=True)
