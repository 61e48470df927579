#!/bin/bash
# Round-3 session F: GPU tests; train-step and forward kernels (packed InterHT score) under a kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/f
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f/prof -o c2 -- \
    python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --sharded-steps 0 > gpurun_out/f/c2.log 2>&1 || { tail -20 gpurun_out/f/c2.log; exit 1; }
grep '^{' gpurun_out/f/c2.log | tail -n 1 | cut -c1-300
echo session-f done
