#!/bin/bash
# Round-6 session I: DMA plane GEMM as the default (eval + TranSparse tests, TS schedule A/B, c5 / c6 bench lines).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06i
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
run tests 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_eval_gpu.py tests/test_transparse_gpu.py tests/test_configs_gpu.py -k 'eval or rank or transparse or c5 or plane'
run probe 600 python3 scripts/ts_sched_probe.py
run c5 600 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline
run c6 600 python3 bench.py --workload c6 --steps 20 --warmup 5 --no-cpu-baseline --train-steps 3
grep '^{' $O/probe.log
echo r06i done
