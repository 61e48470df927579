#!/bin/bash
# Round-6 session T: the tile step's first-candidate L2 prefetch A/B (scripts/prefetch_probe.py), then the planned /
# tile GPU tests on the prefetch build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u scripts/prefetch_probe.py > $O/probe.log 2>&1; rc=$?
echo "probe rc=$rc"; cat $O/probe.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_planned_gpu.py tests/test_tile_gpu.py > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
echo r06t done
