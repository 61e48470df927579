#!/bin/bash
# round 5: TranSparse column-split kernel A/B (library variants from scripts/ab_build.sh): pipeline depth 2/4/6,
# 4- vs 2-wave (128- vs 64-column) split blocks, and the prologue alone (no K loop) — tests, c6 bench, kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
VARS="main=customknowledgegraphembedding_amd/libkge_hip.so dep4=abtmp/dep4/libkge_hip.so dep6=abtmp/dep6/libkge_hip.so w2d2=abtmp/w2d2/libkge_hip.so w2d4=abtmp/w2d4/libkge_hip.so noloop=abtmp/noloop/libkge_hip.so"
for v in $VARS; do
  n=${v%%=*}; lib=${v#*=}
  [ $n = noloop ] && continue
  KGE_HIP_LIB=$R/$lib timeout -k 10 300 python3 -u -m pytest tests/test_transparse_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_$n.log 2>&1 || { tail -30 $O/tests_$n.log; exit 1; }
  echo "tests $n: $(tail -n 1 $O/tests_$n.log)"
done
for v in $VARS; do
  n=${v%%=*}; lib=${v#*=}
  KGE_HIP_LIB=$R/$lib timeout -k 10 300 python3 bench.py --workload c6 --steps 20 --warmup 3 --no-cpu-baseline > $O/c6_$n.json 2> $O/c6_$n.err || { tail -20 $O/c6_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c6_$n.json')); print('$n', d['value'], d['ms_per_step'])"
  cd /tmp && KGE_HIP_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$n -o run -- python3 $R/bench.py --workload c6 --steps 20 --warmup 3 --no-cpu-baseline > $R/$O/prof_$n.log 2>&1 || exit 1
  cd $R
  python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$n/run_kernel_stats.csv')):
    if 'ts_' in r['Name']: print('$n', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
done
echo r05j done
