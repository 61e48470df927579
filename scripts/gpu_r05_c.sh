#!/bin/bash
# round 5: the changed GPU tests (planned step, forms instead of environment knobs, TranSparse column split,
# RCCL self-checking section), then where the next step's plan is made (tile tail / beside the row reductions /
# standalone) and one mode vs alternating modes at C2, C3, C4
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_planned_gpu.py tests/test_rccl_gpu.py tests/test_tile_gpu.py tests/test_transparse_gpu.py tests/test_eval_gpu.py tests/test_abi.py tests/test_trained_range_gpu.py "tests/test_configs_gpu.py::test_c2_xcd_phases_bitwise" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for wl in c2 c3 c4; do
  timeout -k 10 200 python -u scripts/plan_probe.py $wl >> $O/probe.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
done
cat $O/probe.json
timeout -k 10 300 python -u bench.py --workload c6 --steps 20 --warmup 3 > $O/bench_c6.json 2> $O/bench_c6.err || { tail -20 $O/bench_c6.err; exit 1; }
cat $O/bench_c6.json
timeout -k 10 200 python -u scripts/stagger_probe.py > $O/stagger.json 2>> $O/probe.err || exit 1
cat $O/stagger.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/plan_probe.py c2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c6 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c6 --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof_c6.log 2>&1 || exit 1
