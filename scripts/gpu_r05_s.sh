#!/bin/bash
# round 5: kge_eval_query_planes (the query rows written as bf16 planes, no separate split) + full-size every-row
# C3 / C4 parity: eval tests, the C3/C4 every-row tests, the C5 bench line and kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_eval_gpu.py tests/test_abi.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_eval.log 2>&1 || { tail -40 $O/tests_eval.log; exit 1; }
echo "tests eval: $(tail -n 1 $O/tests_eval.log)"
timeout -k 10 300 python3 bench.py --workload c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c5 -o run -- python3 $R/bench.py --workload c5 --steps 50 --warmup 5 --no-cpu-baseline > $R/$O/prof_c5.log 2>&1 || exit 1
cd $R && python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_c5/run_kernel_stats.csv')):
    print('c5', r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
timeout -k 10 900 python3 -u -m pytest "tests/test_configs_gpu.py::test_c3_every_row_full_size" "tests/test_configs_gpu.py::test_c4_every_row_full_size" -m gpu -v -x -p no:cacheprovider --timeout 600 --timeout-method thread --durations=5 > $O/tests_rows.log 2>&1 || { tail -40 $O/tests_rows.log; exit 1; }
tail -8 $O/tests_rows.log
echo r05s done
