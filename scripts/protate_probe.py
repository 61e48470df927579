"""pRotatE scoring time (kge_step_forward, both modes alternating) at C2's shape with a pRotatE model of d = 1000:
events over 50 steps after 10 warmup; prints us per step. Used for the hardware-sin A/B (scripts/gpu_r04_v.sh)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import customknowledgegraphembedding_amd as kge  # noqa: E402
from customknowledgegraphembedding_amd import ops  # noqa: E402
from customknowledgegraphembedding_amd._lib import FN_IDS  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    E, R, d, B, N = 40943, 11, 1000, 512, 256
    m = kge.TFKGEModel("pRotatE", E, R, d, 24.0, device=dev, seed=0)
    g = np.random.RandomState(0)
    batches = [(torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)).to(dev),
                torch.from_numpy(g.randint(E, size=(B, N))).to(dev)) for _ in range(4)]
    ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()

    def step(i):
        pos, neg = batches[i % 4]
        return ops.step_forward_raw(FN_IDS["pRotatE"], i % 2, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f,
                                    m._range_f, float(m.modulus.detach().reshape(-1)[0]))
    for i in range(10):
        step(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(50):
        step(i)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"pRotatE_step_us": e0.elapsed_time(e1) * 1e3 / 50}), flush=True)


if __name__ == "__main__":
    main()
