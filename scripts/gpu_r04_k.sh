#!/bin/bash
# Round 4: the tile kernel with the query ids read in the relation sort (no dependent id load before the query
# rows): parity, C2 / C3 / C4 kernel traces, and the C2 setup levels (KGE_TILE_DRY, profiling-knob build).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
run pytest_tile 600 python3 -u -m pytest tests/test_tile_gpu.py tests/test_configs_gpu.py tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_tile.log
for w in c2 c4 c3; do
  AB="--workload $w --steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
  run ${w} 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w} -o run -- python3 bench.py $AB
done
AB="--steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
for d in 1 2 4; do
  run dry$d 300 env KGE_HIP_LIB=$R/abtmp/prof/libkge_hip.so KGE_TILE_DRY=$d rocprofv3 --kernel-trace --stats --output-format csv -d $O/dry$d -o run -- python3 bench.py $AB
done
echo r04k done
