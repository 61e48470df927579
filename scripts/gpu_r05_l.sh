#!/bin/bash
# round 5: the plane GEMM's step schedule (KGE_X3P_SCHED: 0 compiler order, 1 the next chunk's LDS stores and global
# loads interleaved one pair per 4 MFMAs, 2 = 1 + s_setprio around the step) — eval tests, C5 bench, kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
VARS="main=customknowledgegraphembedding_amd/libkge_hip.so s1=abtmp/s1/libkge_hip.so s2=abtmp/s2/libkge_hip.so"
for v in $VARS; do
  n=${v%%=*}; lib=${v#*=}
  KGE_HIP_LIB=$R/$lib timeout -k 10 300 python3 -u -m pytest tests/test_eval_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_$n.log 2>&1 || { tail -30 $O/tests_$n.log; exit 1; }
  echo "tests $n: $(tail -n 1 $O/tests_$n.log)"
done
for i in 1 2; do
for v in $VARS; do
  n=${v%%=*}; lib=${v#*=}
  KGE_HIP_LIB=$R/$lib timeout -k 10 300 python3 bench.py --workload c5 --no-cpu-baseline > $O/c5_$n$i.json 2> $O/c5_$n$i.err || { tail -20 $O/c5_$n$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$n$i.json')); print('$n$i', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])"
done
done
for v in $VARS; do
  n=${v%%=*}; lib=${v#*=}
  cd /tmp && KGE_HIP_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$n -o run -- python3 $R/bench.py --workload c5 --no-cpu-baseline > $R/$O/prof_$n.log 2>&1 || exit 1
  cd $R && python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$n/run_kernel_stats.csv')):
    if 'gemm' in r['Name'] or 'split3' in r['Name']: print('$n', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
done
echo r05l done
