"""Round 6: the plane GEMM's two forms at C5's shape (4 096 queries x 14 951 entities, K = 1 000 DistMult and
2 000 ComplEx), same process, events around 10 calls, 3 rounds interleaved: form 1 gemm_nt_x3p_kernel (both operands
staged through LDS per 16-k chunk), form 2 gemm_nt_x3d_kernel (B fragments straight into registers, A staged per
32 k), form 3 the staged form with 256 x 192 tiles, form 4 both operands staged by LDS-DMA copies (three stages). C compared bitwise. Fraction of the bf16 dense peak (2.5 PFLOP/s) on the six executed products.
Usage: python scripts/gemm_form_probe.py"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from customknowledgegraphembedding_amd import _lib, evaluate  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream().cuda_stream
M, N = 4096, 14951
for K in (1000, 2000):
    g = torch.Generator().manual_seed(K)
    A = torch.randn(M, K, generator=g).to(dev)
    Bm = torch.randn(N, K, generator=g).to(dev)
    ap, bp = evaluate.split_planes(A), evaluate.split_planes(Bm)
    res = {"M": M, "N": N, "K": K, "form1_us": [], "form2_us": [], "form3_us": [], "form4_us": []}
    outs = {}
    for _ in range(3):
        for form in (1, 2, 3, 4):
            f = _lib.forms(gemm_form=form)
            C = torch.empty(M, N, device=dev)

            def call():
                assert lib.kge_gemm_nt_bf16x3_planes_ex(ap.data_ptr(), M, bp.data_ptr(), N, K, C.data_ptr(), N, M, N,
                                                        ctypes.addressof(f), st) == 0
            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call()
            e1.record()
            torch.cuda.synchronize()
            res[f"form{form}_us"].append(round(e0.elapsed_time(e1) / 10 * 1e3, 1))
            outs[form] = C.clone()
    res["bitwise_equal"] = all(bool(torch.equal(outs[1], outs[f])) for f in (2, 3, 4))
    flop = 2.0 * M * N * ((K + 15) // 16 * 16) * 6
    for form in (1, 2, 3, 4):
        res[f"form{form}_frac_bf16_peak"] = round(flop / (min(res[f"form{form}_us"]) * 1e-6) / 2.5e15, 3)
    print(json.dumps(res), flush=True)
