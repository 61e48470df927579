#!/bin/bash
# Round 4, session E: the native executor's device timeline with the collectives on the step's own stream
# (KGE_EXEC_ONE_STREAM) against a communication stream, K = 1 and 2; its tests; host cost.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 40 "$O/$n.log"; exit $rc; fi
}
run pytest_native 300 python3 -u -m pytest tests/test_native_exec_gpu.py tests/test_rccl_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
tail -n 1 $O/pytest_native.log
for cfg in "2 0" "1 0" "2 1" "1 1"; do
  set -- $cfg
  n=tl_k$1_one$2
  run $n 300 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o run -- python3 scripts/native_timeline.py $1 40 $2
  python3 scripts/native_timeline.py --analyze $O/$n > $O/$n.json; echo "$n"; head -4 $O/$n.json
done
run host_probe1 300 env KGE_SHARD_ONE_STREAM=1 python3 scripts/shard_host_probe.py 8 20
grep '^{' $O/host_probe1.log | head -1
echo r04e done
