#!/bin/bash
# Round-3 session D: GPU tests, rank-0 probe under a kernel trace (device durations per kernel).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/probe/prof -o probe -- \
    python3 scripts/shard_probe.py --chunks 1,4 --reps 10 > gpurun_out/probe/prof.log 2>&1 || { tail -20 gpurun_out/probe/prof.log; exit 1; }
tail -n 1 gpurun_out/probe/prof.log
f=$(find gpurun_out/probe/prof -name '*kernel_stats.csv' | head -n 1)
cut -d, -f1-4 "$f" | head -n 25
echo session-d done
