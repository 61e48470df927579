#!/bin/bash
# Round-5 final measurement: GPU tests, smoke, two-process step, PMC passes (c2 c3 c4 c6) summarised into
# gpurun_out/pmc/pmc_<w>.json, then the bench lines c2..c6 (which read the committed PMC summaries only
# when they match the library's sources: the copies are made by the caller afterwards, so this run's lines
# carry traffic from gpurun_out via KGE_PMC_DIR), the kernel traces of every workload and the native
# executor's host cost.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/final5
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$O/$n.log"; exit $rc; fi
}
run bench_c2 600 python3 bench.py
for wl in c3 c4 c5 c6; do run bench_$wl 600 python3 bench.py --workload $wl; done
run prof_c2 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --sharded-steps 0
run prof_c3 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --workload c3 --steps 50 --warmup 5 --no-cpu-baseline --sharded-steps 0 --train-steps 0
for wl in c4 c5 c6; do
  run prof_$wl 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- \
      python3 bench.py --workload $wl --steps 50 --warmup 5 --no-cpu-baseline --sharded-steps 0 --train-steps 0
done
run host_probe 300 python3 scripts/shard_host_probe.py 8 20
echo final5 part B done
