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
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_gpu.log
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
run two_proc 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 scripts/shard_two_proc.py
for W in ${PMC_WLS:-c2 c3 c4 c6}; do
  bash scripts/pmc.sh "$W" > $O/pmc_$W.log 2>&1 || { tail -5 $O/pmc_$W.log; exit 1; }
  python3 scripts/pmc_summary.py "gpurun_out/pmc/$W" "gpurun_out/pmc/pmc_$W.json" > "gpurun_out/pmc/$W/summary.txt" 2>&1 || exit 1
  echo "pmc $W done"
done
echo final5 part A done
