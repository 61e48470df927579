#!/bin/bash
# Round 4: C4 tile sweep with more DistMult candidate rows in flight per wave (a ring of 4 or 6 items instead of
# 2; abtmp/deep4, abtmp/deep6) against the shipped library: tile / config tests on deep4, C4 kernel traces.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
run pytest_deep 600 env KGE_HIP_LIB=$R/abtmp/deep4/libkge_hip.so python3 -u -m pytest tests/test_tile_gpu.py tests/test_configs_gpu.py tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_deep.log
AB="--workload c4 --steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
for v in base deep4 deep6 base2 deep42 deep62; do
  L=""
  case $v in deep4*) L="env KGE_HIP_LIB=$R/abtmp/deep4/libkge_hip.so";; deep6*) L="env KGE_HIP_LIB=$R/abtmp/deep6/libkge_hip.so";; esac
  run c4_$v 300 $L rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_$v -o run -- python3 bench.py $AB
done
echo r04u done
