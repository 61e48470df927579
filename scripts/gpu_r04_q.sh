#!/bin/bash
# Round 4: is the row-reduction launch (neg_rows_kernel) bound by its libm exp / log? A/B against a build whose
# reduction uses the hardware exp / log (abtmp/rowsfast, -DKGE_ROWS_FAST=1; timing only, not bitwise).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
F=$R/abtmp/rowsfast/libkge_hip.so
for w in c2 c4; do
  AB="--workload $w --steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
  for v in base fast base2 fast2; do
    if [ "${v#fast}" != "$v" ]; then L="env KGE_HIP_LIB=$F"; else L=""; fi
    run ${w}_$v 300 $L rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_$v -o run -- python3 bench.py $AB
  done
done
echo r04q done
