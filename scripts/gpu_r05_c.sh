#!/bin/bash
# round 5: where the next step's plan is made (tile tail / beside the row reductions / standalone) at C2, C3, C4
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_planned_gpu.py tests/test_rccl_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for wl in c2 c3 c4; do
  timeout -k 10 200 python -u scripts/plan_probe.py $wl >> $O/probe.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
done
cat $O/probe.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/plan_probe.py c2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
