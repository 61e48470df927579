#!/bin/bash
# Round-6 session M: eval tests with the two-stream rank pipeline and the empty-filter fix, C5 two streams against one (same box, alternating).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06m
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi  # 1: test failures (go on); anything else: stop
}
run tests 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_eval_gpu.py tests/test_configs_gpu.py tests/test_run_gpu.py -k "eval or rank or c5 or run"
tail -n 3 $O/tests.log
run c5 600 python3 bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline
run c5_1 600 env KGE_BENCH_EVAL_SPLIT=planes1 python3 bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline
run c5b 600 python3 bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline
run c5_1b 600 env KGE_BENCH_EVAL_SPLIT=planes1 python3 bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline
run prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline
echo r06m done
