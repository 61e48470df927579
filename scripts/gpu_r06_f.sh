#!/bin/bash
# Round-6 session F: TranSparse head-batch staging among the MFMAs (tests, A/B at c6, c6 bench + rocprof).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06f
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
run tests 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_transparse_gpu.py
run probe 600 python3 scripts/ts_sched_probe.py
run bench 600 python3 bench.py --workload c6 --steps 20 --warmup 5 --no-cpu-baseline --train-steps 3
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 bench.py --workload c6 --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0
grep '^{' $O/probe.log $O/bench.log
echo r06f done
