#!/bin/bash
# round 5: planned tile step (kge_step_forward_planned) + trained-range parity; C2 bench planned vs unplanned
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_planned_gpu.py tests/test_trained_range_gpu.py tests/test_tile_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
KGE_BENCH_UNPLANNED=1 timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $O/bench_c2_unplanned.json 2>> $O/bench_c2.err || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -3
