#!/bin/bash
# round 5: every row of full-size C3 and C4, both modes, scores and row outputs against the fp64 oracle
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest "tests/test_configs_gpu.py::test_c3_every_row_full_size" "tests/test_configs_gpu.py::test_c4_every_row_full_size" "tests/test_configs_gpu.py::test_c2_every_row_full_size" -m gpu -v -x -p no:cacheprovider --timeout 170 --timeout-method thread --durations=5 2>&1 | tee $O/tests_rows.log
