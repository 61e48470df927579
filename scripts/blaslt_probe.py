"""Round 6 probe: what the vendor GEMM (torch.mm -> hipBLASLt / rocBLAS) sustains on the plane GEMM's work written as
ONE bf16 GEMM over the six products concatenated along K (A' = [a2 a1 a0 a1 a0 a0], B' = [b0 b1 b2 b0 b1 b0], K' =
6 x 1008), fp32 output where torch offers it, at C5's shape (4 096 x 14 951). Events around 10 calls, best of 3.
Usage: python scripts/blaslt_probe.py"""
import json

import torch

dev = torch.device("cuda", 0)
M, N, K = 4096, 14951, 6 * 1008
A = torch.randn(M, K, device=dev).bfloat16()
B = torch.randn(N, K, device=dev).bfloat16()
flop = 2.0 * M * N * K


def timeit(call):
    call()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            call()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
    return round(best, 1)


res = {"M": M, "N": N, "K_concat": K}
res["bf16_out_us"] = timeit(lambda: torch.mm(A, B.t()))
res["bf16_out_frac_bf16_peak"] = round(flop / (res["bf16_out_us"] * 1e-6) / 2.5e15, 3)
try:
    res["f32_out_us"] = timeit(lambda: torch.mm(A, B.t(), out_dtype=torch.float32))
    res["f32_out_frac_bf16_peak"] = round(flop / (res["f32_out_us"] * 1e-6) / 2.5e15, 3)
except Exception as e:  # noqa: BLE001
    res["f32_out_error"] = repr(e)[:200]
Bt = B.t().contiguous()
res["bf16_out_nn_us"] = timeit(lambda: torch.mm(A, Bt))
print(json.dumps(res), flush=True)
