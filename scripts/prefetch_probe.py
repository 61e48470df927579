"""Round 6: the planned tile step with each wave's first candidate row pulled into L2 before the query build
(KGE_TILE_PREFETCH=1, the library) against a build without it (-DKGE_TILE_PREFETCH=0, scripts/ab_build.sh into
abtmp/nopf). One child process per library and turn, libraries alternating (A B A B); in each, C2 / C3 / C4
planned steps (bench.StepRunner, alternating modes and sweep), device us per step over 60 steps after 20 warmup,
3 rounds. Usage: python scripts/prefetch_probe.py"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys, torch
sys.path.insert(0, ROOT)
import bench
from customknowledgegraphembedding_amd import ops
from customknowledgegraphembedding_amd._lib import FN_IDS
bench.ops = ops
dev = torch.device("cuda", 0)
res = {"lib": LIB}
for wl in ("c2", "c3", "c4"):
    w = bench.WORKLOADS[wl]
    m, batches = bench.make_inputs(w, 0, dev)
    r = bench.StepRunner(m, batches, FN_IDS[w["fn"]], planned=True)
    k, out = 0, []
    for rnd in range(3):
        for i in range(20):
            r(k); k += 1
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(60):
            r(k); k += 1
        e1.record()
        torch.cuda.synchronize()
        out.append(round(e0.elapsed_time(e1) / 60 * 1e3, 2))
    res[wl] = out
    del m, batches, r
    torch.cuda.empty_cache()
print("RESULT " + json.dumps(res), flush=True)
'''
libs = [os.path.join(ROOT, "customknowledgegraphembedding_amd", "libkge_hip.so"),
        os.path.join(ROOT, "abtmp", "nopf", "libkge_hip.so")]
for turn in range(2):
    for lp in libs:
        env = dict(os.environ, KGE_HIP_LIB=lp)
        code = f"ROOT = {ROOT!r}\nLIB = {os.path.relpath(lp, ROOT)!r}\n" + CHILD
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=400)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
        print(line[0][7:] if line else json.dumps({"lib": lp, "rc": p.returncode, "err": p.stderr[-800:]}), flush=True)
