#!/bin/bash
# Round 4: tile setup A/B — the relation sort's prefix summed in registers, the relation slots by one ballot,
# and a walk capacity of 17 items per thread (C4 tail-batch: 16 x 1 025 items now walked once).
# base = this tree's build, old = the previous kernels (abtmp/old, built by scripts/ab_build.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
run pytest_tile 600 python3 -u -m pytest tests/test_tile_gpu.py tests/test_configs_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_tile.log
OLD=$R/abtmp/old/libkge_hip.so
for w in c2 c4 c3; do
  AB="--workload $w --steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
  run ${w}_base 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_base -o run -- python3 bench.py $AB
  run ${w}_old 300 env KGE_HIP_LIB=$OLD rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_old -o run -- python3 bench.py $AB
  run ${w}_base2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_base2 -o run -- python3 bench.py $AB
  run ${w}_old2 300 env KGE_HIP_LIB=$OLD rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_old2 -o run -- python3 bench.py $AB
done
echo r04h done
