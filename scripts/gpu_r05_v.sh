#!/bin/bash
# round 5: TranSparse head-batch with M_r split once per call into bf16 planes (ts_mplanes_kernel + x3s<.., true>)
# epilogues): the TranSparse GPU tests, the c6 bench line, the c6 kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_transparse_gpu.py tests/test_abi.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -n 1 $O/tests.log)"
for i in 1 2; do
timeout -k 10 300 python3 bench.py --workload c6 > $O/c6_$i.json 2> $O/c6_$i.err || { tail -20 $O/c6_$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c6_$i.json')); print('c6', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c6 -o run -- python3 $R/bench.py --workload c6 --steps 50 --warmup 5 --no-cpu-baseline --sharded-steps 0 --train-steps 0 > $R/$O/prof_c6.log 2>&1 || exit 1
cd $R && python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_c6/run_kernel_stats.csv')):
    print('c6', r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
timeout -k 10 200 python3 -u scripts/ts_planes_probe.py > $O/planes_probe.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/planes_probe.json
echo r05v done
