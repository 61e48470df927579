#!/bin/bash
# Round-6 session K: the whole GPU suite and smoke on the LDS-DMA plane GEMM / scheduled TranSparse build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06k
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
run tests 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
tail -n 3 $O/tests.log
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
echo r06k done
