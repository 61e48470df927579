#!/bin/bash
# Round-3 session E: GPU tests, rank-0 probe under a kernel trace, default bench line (C2 + row-sharded + sim).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/probe/prof -o probe -- \
    python3 scripts/shard_probe.py --chunks 1,2,4 --reps 10 > gpurun_out/probe/prof.log 2>&1 || { tail -20 gpurun_out/probe/prof.log; exit 1; }
tail -n 1 gpurun_out/probe/prof.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-600
echo session-e done
