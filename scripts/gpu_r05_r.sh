#!/bin/bash
# round 5: every row of full-size C3 and C4, both modes, scores and row outputs against the fp64 oracle
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest "tests/test_configs_gpu.py::test_c3_every_row_full_size" "tests/test_configs_gpu.py::test_c4_every_row_full_size" -m gpu -v -x -p no:cacheprovider --timeout 600 --timeout-method thread --durations=5 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -12 $O/tests.log
