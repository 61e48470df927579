#!/bin/bash
# round 5: trained-range parity (range-reduced hardware sin / cos, series log1p in the row reductions)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_trained_range_gpu.py tests/test_parity_gpu.py tests/test_tile_gpu.py > gpurun_out/r05a/tests.log 2>&1
rc=$?
tail -5 gpurun_out/r05a/tests.log
exit $rc
