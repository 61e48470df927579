#!/bin/bash
# GPU tests, then a kernel-trace profile of the bench's train-step side measurement.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python3 -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider -x > gpurun_out/all.log 2>&1; rc=$?; tail -2 gpurun_out/all.log
[ $rc -ge 124 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab/t -o run -- python3 $R/bench.py --no-cpu-baseline --sharded-steps 0 --steps 5 --train-steps 20 > gpurun_out/ab_t.json 2>/dev/null || exit $?
echo ok
