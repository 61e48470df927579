"""Times the reference's literal call path at C2: model(((pos, neg), mode)) then model(((pos, neg), 3))
(supervisor.py:17-18 as two calls: kge_score_indexed + kge_neg_reduce, then the single-mode call)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import customknowledgegraphembedding_amd as kge  # noqa: E402

E, R, d, B, N = 40943, 11, 1000, 512, 256
m = kge.TFKGEModel("InterHT", E, R, d, 24.0, double_entity_embedding=True, triple_relation_embedding=True,
                   device="cuda", seed=0)
g = np.random.RandomState(1)
pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)).cuda()
neg = torch.from_numpy(np.random.RandomState(2).randint(E, size=(B, N))).cuda()
with torch.no_grad():
    for i in range(5):
        m(((pos, neg), i % 2)), m(((pos, neg), 3))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(20):
        m(((pos, neg), i % 2)), m(((pos, neg), 3))
    e1.record()
    torch.cuda.synchronize()
print(f"two-call step {e0.elapsed_time(e1) / 20 * 1e3:.1f} us")
