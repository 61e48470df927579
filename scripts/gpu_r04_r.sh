#!/bin/bash
# Round 4: forward row reductions on the hardware exp / log (abtmp/rrhw, KGE_RR_HW=1): the whole GPU suite on
# it, then C4 / C2 kernel traces against the shipped library, alternating.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04r
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
F=$R/abtmp/rrhw/libkge_hip.so
run pytest_rrhw 900 env KGE_HIP_LIB=$F python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_rrhw.log
for w in c4 c2; do
  AB="--workload $w --steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
  for v in base hw base2 hw2; do
    if [ "${v#hw}" != "$v" ]; then L="env KGE_HIP_LIB=$F"; else L=""; fi
    run ${w}_$v 300 $L rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_$v -o run -- python3 bench.py $AB
  done
done
echo r04r done
