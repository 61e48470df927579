#!/bin/bash
# Round-6 session C: the fused-rank tests first, the GPU suite and smoke on this build, the C2 PMC passes of this
# build (gpurun_out/pmc/pmc_c2.json), the headline line reading them (KGE_PMC_DIR), C5 on the fused ranks against
# the score-matrix path (same box), and the kernel traces of C2 and C5.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi  # 1: test failures (go on); anything else: stop
}
run new 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_eval_gpu.py tests/test_configs_gpu.py -k 'rank_planes or ranks_from_planes or c5'
run tests 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
tail -n 3 $O/tests.log
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
bash scripts/pmc.sh c2 > $O/pmc_c2.log 2>&1 || { tail -5 $O/pmc_c2.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc/c2 gpurun_out/pmc/pmc_c2.json > gpurun_out/pmc/c2/summary.txt 2>&1 || exit 1
run bench_c2 600 env KGE_PMC_DIR=gpurun_out/pmc python3 bench.py --steps 20 --warmup 5
run bench_c5 600 python3 bench.py --workload c5
run bench_c5_s 600 env KGE_BENCH_EVAL_SPLIT=planes_s python3 bench.py --workload c5
run prof_c2 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --sharded-steps 0
run prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
    python3 bench.py --workload c5 --steps 50 --warmup 5
tail -n 1 $O/bench_c2.log | cut -c1-400
for f in bench_c5 bench_c5_s; do tail -n 1 $O/$f.log | cut -c1-300; done
echo r06c done
