#!/bin/bash
# Round-6 final session P (frozen library): C5 (FB15k filtered ranks, two streams) and c6 (TranSparse) PMC passes,
# bench lines and kernel traces on this build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06p
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
for W in c5 c6; do
  bash scripts/pmc.sh $W > $O/pmc_$W.log 2>&1 || { tail -5 $O/pmc_$W.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/pmc/$W gpurun_out/pmc/pmc_$W.json > gpurun_out/pmc/$W/summary.txt 2>&1 || exit 1
  run bench_$W 600 python3 bench.py --workload $W --steps 40 --warmup 5
  run prof_$W 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$W -o run -- \
      python3 bench.py --workload $W --steps 40 --warmup 5 --no-cpu-baseline --train-steps 0
done
echo r06p done
