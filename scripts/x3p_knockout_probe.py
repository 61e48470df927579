"""Round 6: step-cost breakdown of the two staged bf16x3 MFMA kernels by knock-out builds (scripts/ab_build.sh with
-DKGE_X3P_KO=<bits> for the plane GEMM gemm_nt_x3p_kernel, -DKGE_TS_KO=<bits> for the TranSparse head-batch
ts_fwd_x3s_kernel; bit 0 no per-chunk barrier, bit 1 no LDS stores, bit 2 no global loads, bit 3 (GEMM) no fragment
reads). Results are wrong in every knock-out build by design; only the device time is read. One child process per
library (KGE_HIP_LIB), events around 10 calls, best of 3 rounds.
Usage: python scripts/x3p_knockout_probe.py [lib ...]   (default: the in-tree library and abtmp/*/libkge_hip.so)"""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes, json, sys
import numpy as np, torch
sys.path.insert(0, ROOT)
from customknowledgegraphembedding_amd import _lib, evaluate, ops
from customknowledgegraphembedding_amd.model import TFKGEModel
lib = _lib.load()
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream().cuda_stream
def timeit(call):
    call(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            call()
        e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
    return round(best, 1)
res = {"lib": LIB}
M, N, K = 4096, 14951, 1000
g = torch.Generator().manual_seed(K)
A = torch.randn(M, K, generator=g).to(dev); Bm = torch.randn(N, K, generator=g).to(dev)
ap, bp = evaluate.split_planes(A), evaluate.split_planes(Bm)
C = torch.empty(M, N, device=dev)
f = _lib.forms(gemm_form=1)
res["gemm_x3p_us"] = timeit(lambda: lib.kge_gemm_nt_bf16x3_planes_ex(ap.data_ptr(), M, bp.data_ptr(), N, K, C.data_ptr(),
                                                                    N, M, N, ctypes.addressof(f), st))
del A, Bm, ap, bp, C
E, R, d, B, Nn = 40943, 11, 500, 512, 256
m = TFKGEModel("TranSparse", E, R, d, 12.0, device="cuda", seed=0)
ent, rel, W, mask = m.entity_embedding.detach(), m.relation_embedding.detach(), m.W.detach(), m.mask
r = np.random.RandomState(1)
pos = torch.from_numpy(np.stack([r.randint(E, size=B), r.randint(R, size=B), r.randint(E, size=B)], 1)).cuda()
neg = torch.from_numpy(np.random.RandomState(2).randint(E, size=(B, Nn))).cuda()
Mp = ops.transparse_premul(W, mask)
for form in (0, 2):
    res[f"ts_form{form}_us"] = timeit(lambda: ops.transparse_score_raw(0, ent, rel, W, mask, pos, neg, 12.0, M=Mp,
                                                                       split=True, forms=dict(transparse_form=form)))
print("RESULT " + json.dumps(res), flush=True)
'''

libs = sys.argv[1:] or ([os.path.join(ROOT, "customknowledgegraphembedding_amd", "libkge_hip.so")] +
                        sorted(glob.glob(os.path.join(ROOT, "abtmp", "*", "libkge_hip.so"))))
for lp in libs:
    env = dict(os.environ, KGE_HIP_LIB=lp)
    code = f"ROOT = {ROOT!r}\nLIB = {os.path.relpath(lp, ROOT)!r}\n" + CHILD
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
    print(line[0][7:] if line else json.dumps({"lib": lp, "rc": p.returncode, "err": p.stderr[-600:]}), flush=True)
