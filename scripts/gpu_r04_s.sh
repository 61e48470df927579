#!/bin/bash
# Round 4: C5 eval GEMM with the columns past the last whole round of 256-tiles on 128-tiles (abtmp/tail) against
# the shipped single launch: bitwise tests, then C5 kernel traces alternating.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
F=$R/abtmp/tail/libkge_hip.so
run pytest_tail 600 env KGE_HIP_LIB=$F python3 -u -m pytest tests/test_eval_gpu.py tests/test_configs_gpu.py -k "gemm or c5 or eval" -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_tail.log
AB="--workload c5 --steps 50 --warmup 5 --no-cpu-baseline"
for v in base tail base2 tail2; do
  if [ "${v#tail}" != "$v" ]; then L="env KGE_HIP_LIB=$F"; else L=""; fi
  run c5_$v 300 $L rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_$v -o run -- python3 bench.py $AB
done
echo r04s done
