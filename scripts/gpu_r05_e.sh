#!/bin/bash
# round 5: the plan group with its positives loaded beside the walk; C2 default bench line and rocprof
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_planned_gpu.py tests/test_tile_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u scripts/plan_probe.py c2 > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.json
timeout -k 10 600 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $GRAFT_REPO_ROOT/$O/prof_c2.log 2>&1 || exit 1
