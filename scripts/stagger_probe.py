"""Round-5 A/B: the SIMD-partner stagger (waves 4-7 store the next chunk before multiplying) in the eval GEMM
(gemm_nt_x3s_kernel, C5 shape 4096 x 14951 x 1000) and the TranSparse head-batch forward (ts_fwd_x3s_kernel, c6
shape); the TranSparse single-mode rows split over 128-column ranges (ts_fwd_x3g_kernel<4, 1> + finish) against
one block per relation chunk. Device time per launch, forms interleaved, 3 rounds of 10 launches each.
(The no-stagger forms 2 it compared were removed after this A/B: profiles/r05_stagger_ab.txt.)"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from customknowledgegraphembedding_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.load()
st = torch.cuda.current_stream().cuda_stream


def timed(f, n=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f()
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


res = {}
g = torch.Generator().manual_seed(0)
M, N, K = 4096, 14951, 1000
A = torch.randn(M, K, generator=g).to(dev)
Bm = torch.randn(N, K, generator=g).to(dev)
C = torch.empty(M, N, device=dev)
forms = {k: _lib.forms(gemm_form=v) for k, v in (("stagger", 0), ("plain", 2))}
for k in forms:
    res["gemm_" + k] = []
for _ in range(3):
    for k, f in forms.items():
        res["gemm_" + k].append(timed(lambda: lib.kge_gemm_nt_bf16x3_ex(A.data_ptr(), K, Bm.data_ptr(), K, C.data_ptr(), N,
                                                                        M, N, K, ctypes.addressof(f), st)))
E, R, d, B, Nn = 40943, 11, 500, 512, 256
ent = (torch.rand(E, d, generator=g) - 0.5).to(dev)
rel = (torch.rand(R, d, generator=g) - 0.5).to(dev)
W = (torch.rand(R, d, d, generator=g) - 0.5).to(dev)
mask = (torch.rand(R, d, d, generator=g) > 0.5).float().to(dev)
pos = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                   torch.randint(0, E, (B,), generator=g)], 1).to(dev)
neg = torch.randint(0, E, (B, Nn), generator=g).to(dev)
for k in ("ts_head_stagger", "ts_head_plain", "ts_single_split", "ts_single_one"):
    res[k] = []
for _ in range(3):
    res["ts_head_stagger"].append(timed(lambda: ops.transparse_score_raw(0, ent, rel, W, mask, pos, neg, 12.0,
                                                                         forms=dict(transparse_form=0))))
    res["ts_head_plain"].append(timed(lambda: ops.transparse_score_raw(0, ent, rel, W, mask, pos, neg, 12.0,
                                                                       forms=dict(transparse_form=2))))
    res["ts_single_split"].append(timed(lambda: ops.transparse_score_raw(3, ent, rel, W, mask, pos, neg, 12.0)))
    res["ts_single_one"].append(timed(lambda: ops.transparse_score_raw(3, ent, rel, W, mask, pos, neg, 12.0,
                                                                       split=False)))
print(json.dumps({k: [round(x, 2) for x in v] for k, v in res.items()}), flush=True)
