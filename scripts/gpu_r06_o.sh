#!/bin/bash
# Round-6 final session O (frozen library): PMC passes and bench lines of C3 (FB15k-237 RotatE) and C4 (YAGO3-10
# DistMult) on this build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for W in c3 c4; do
  bash scripts/pmc.sh $W > $O/pmc_$W.log 2>&1 || { tail -5 $O/pmc_$W.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/pmc/$W gpurun_out/pmc/pmc_$W.json > gpurun_out/pmc/$W/summary.txt 2>&1 || exit 1
  run bench_$W 600 env KGE_PMC_DIR=gpurun_out/pmc python3 bench.py --workload $W --steps 50 --warmup 5
done
echo r06o done
