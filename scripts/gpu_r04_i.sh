#!/bin/bash
# Round 4: (1) parity of this build's tile setup (walk capacity by wave count), (2) the train-forward order
# question: partial-state traffic probe + the plain forward in each order + the train step with
# real and L2-hot gathers, each variant in its own rocprofv3 kernel-trace process.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
# run pytest_tile 600 python3 -u -m pytest tests/test_tile_gpu.py tests/test_configs_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
# tail -n 1 $O/pytest_tile.log
# run partial 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/partial -o run -- ./tools/partial_merge_probe 512 1000 50
# cat $O/partial.log | grep '^{'
for v in train_m2048 train_m16384; do
  run $v 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 scripts/train_order_probe.py $v 100
  grep '^{' $O/$v.log
done
echo r04i done
