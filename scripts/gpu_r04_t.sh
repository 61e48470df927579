#!/bin/bash
# Round 4: RotatE query build on the hardware sin / cos (abtmp/rothw, KGE_ROT_HW=1: the C3 tile kernel 168 VGPRs
# + 24 B of scratch -> 115, no scratch): the whole GPU suite on it, then C3 kernel traces against the shipped
# library at 12 waves, and the variant at 16 waves (KGE_TILE_WAVES=16, spill-free now).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04t
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
F=$R/abtmp/rothw/libkge_hip.so
run pytest_rothw 900 env KGE_HIP_LIB=$F python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_rothw.log
AB="--workload c3 --steps 100 --warmup 10 --train-steps 20 --sharded-steps 0 --no-cpu-baseline"
for v in base hw base2 hw2 hw16; do
  L=""
  case $v in hw|hw2) L="env KGE_HIP_LIB=$F";; hw16) L="env KGE_HIP_LIB=$F KGE_TILE_WAVES=16";; esac
  run c3_$v 300 $L rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3_$v -o run -- python3 bench.py $AB
done
echo r04t done
