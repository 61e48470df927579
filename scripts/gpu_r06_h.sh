#!/bin/bash
# Round-6 session H: plane GEMM with LDS-DMA staging (tests, GEMM and rank A/B, C5 bench + rocprof).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06h
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
run tests 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_eval_gpu.py -k 'b_direct or rank_planes'
run gemm 600 python3 scripts/gemm_form_probe.py
run rank 600 python3 scripts/rank_form_probe.py
grep '^{' $O/gemm.log $O/rank.log
echo r06h done
