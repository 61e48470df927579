#!/bin/bash
# Round 4: what the C2 tile setup's query-build stage waits on (KGE_TILE_DRY=2, profiling-knob builds):
# prof = shipped order; exp1 = no walk before the query build; exp2 = query rows read as zeros (no traffic).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
AB="--steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
for v in prof exp1 exp2 prof; do
  for d in 1 2; do
    run ${v}_dry$d 300 env KGE_HIP_LIB=$R/abtmp/$v/libkge_hip.so KGE_TILE_DRY=$d rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_dry$d -o run -- python3 bench.py $AB
  done
done
echo r04l done
