#!/bin/bash
# Round-6 session D: the fused-rank and C5 tests after the pair-kernel change, C5 fused vs score-matrix lines, and
# the C5 kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06d
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
run new 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_eval_gpu.py tests/test_configs_gpu.py -k 'rank_planes or ranks_from_planes or c5 or test_step'
run bench_c5 600 python3 bench.py --workload c5
run bench_c5_s 600 env KGE_BENCH_EVAL_SPLIT=planes_s python3 bench.py --workload c5
run prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
    python3 bench.py --workload c5 --steps 50 --warmup 5
for f in bench_c5 bench_c5_s; do tail -n 1 $O/$f.log | cut -c1-250; done
echo r06d done
