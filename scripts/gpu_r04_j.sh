#!/bin/bash
# Round 4: the C2 tile kernel's setup, stage by stage (KGE_TILE_DRY levels: 1 = relation sort, 2 = + query build,
# 3 = + walk histogram, 4 = + scan / scatter; NOSORT + DRY 1 = an almost empty launch), kernel-trace averages.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
export KGE_HIP_LIB=$R/abtmp/prof/libkge_hip.so  # the DRY / NOSORT knobs need -DKGE_PROFILING_KNOBS
AB="--steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
run empty 300 env KGE_TILE_DRY=1 KGE_TILE_NOSORT=1 rocprofv3 --kernel-trace --stats --output-format csv -d $O/empty -o run -- python3 bench.py $AB
for d in 1 2 3 4; do
  run dry$d 300 env KGE_TILE_DRY=$d rocprofv3 --kernel-trace --stats --output-format csv -d $O/dry$d -o run -- python3 bench.py $AB
done
run full 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/full -o run -- python3 bench.py $AB
echo r04j done
