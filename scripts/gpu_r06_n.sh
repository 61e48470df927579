#!/bin/bash
# Round-6 final session N (frozen library): the whole GPU suite and smoke, the C2 PMC passes of this build
# (gpurun_out/pmc/pmc_c2.json), the default bench line reading them (KGE_PMC_DIR), the C2 kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06n
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
run tests 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
tail -n 3 $O/tests.log
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
bash scripts/pmc.sh c2 > $O/pmc_c2.log 2>&1 || { tail -5 $O/pmc_c2.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc/c2 gpurun_out/pmc/pmc_c2.json > gpurun_out/pmc/c2/summary.txt 2>&1 || exit 1
run bench_c2 600 env KGE_PMC_DIR=gpurun_out/pmc python3 bench.py
run prof_c2 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --sharded-steps 0
echo r06n done
