#!/bin/bash
# Round-6 session V: the C2 step's warm-up curve from a cold start, with and without a clock-ramping GEMM first.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u scripts/warmup_probe.py 0 1 2 0 1 2 > $O/probe4.log 2>&1; rc=$?
echo "probe rc=$rc"; cat $O/probe4.log | tail -7
echo r06v done
