#!/bin/bash
# Round 4, session B: the native row-sharded executor (kge_comm.hip): its GPU tests (loopback ranks,
# RCCL at world 1), the host cost of one rank-step at W = 8, then the whole GPU suite.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 40 "$O/$n.log"; exit $rc; fi
}
run pytest_native 300 python3 -u -m pytest tests/test_native_exec_gpu.py -v -x -p no:cacheprovider --timeout 120 --timeout-method thread
tail -n 2 $O/pytest_native.log
run pytest_rccl 300 python3 -u -m pytest tests/test_rccl_gpu.py -v -x -p no:cacheprovider --timeout 120 --timeout-method thread
tail -n 2 $O/pytest_rccl.log
run host_probe 300 python3 scripts/shard_host_probe.py 8 20
grep '^{' $O/host_probe.log
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_gpu.log
echo r04b done
