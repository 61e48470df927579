#!/bin/bash
# round 5: plan walk in 32-bit slice math; probe with the plan kernel alone; planned tests
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_planned_gpu.py tests/test_tile_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for wl in c2 c3 c4; do
timeout -k 10 200 python -u scripts/plan_probe.py $wl >> $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
done
cat $O/probe.json
