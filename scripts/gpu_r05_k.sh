#!/bin/bash
# round 5: TranSparse forwards with unconditional loads (static wait counts) and a MASK template flag: depth and split-width A/B
# 4- vs 2-wave (128- vs 64-column) split blocks, and the prologue alone (no K loop) — tests, c6 bench, kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
VARS="main=customknowledgegraphembedding_amd/libkge_hip.so dep4=abtmp/dep4/libkge_hip.so w2d2=abtmp/w2d2/libkge_hip.so w2d4=abtmp/w2d4/libkge_hip.so"
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
echo r05k done
# the eval GEMMs with unconditional loads: tests, C5 bench, kernel trace
timeout -k 10 300 python3 -u -m pytest tests/test_eval_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_eval.log 2>&1 || { tail -30 $O/tests_eval.log; exit 1; }
echo "tests eval: $(tail -n 1 $O/tests_eval.log)"
timeout -k 10 300 python3 bench.py --workload c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
cat $O/c5.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c5 -o run -- python3 $R/bench.py --workload c5 --no-cpu-baseline > $R/$O/prof_c5.log 2>&1 || exit 1
cd $R && python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_c5/run_kernel_stats.csv')):
    print('c5', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
echo r05k eval done
# the tile sweep with unconditional candidate loads: tests, C2/C3/C4 benches (driver form), kernel trace at C2
timeout -k 10 400 python3 -u -m pytest tests/test_tile_gpu.py tests/test_planned_gpu.py tests/test_configs_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_tile.log 2>&1 || { tail -30 $O/tests_tile.log; exit 1; }
echo "tests tile: $(tail -n 1 $O/tests_tile.log)"
for wl in c2 c3 c4; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --sharded-steps 0 > $O/$wl.json 2> $O/$wl.err || { tail -20 $O/$wl.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$wl.json')); print('$wl', d['value'], d['ms_per_step'], (d.get('train_step') or {}).get('ms_per_step'))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c2 -o run -- python3 $R/scripts/plan_probe.py c2 > $R/$O/prof_c2.log 2>&1 || exit 1
cd $R && python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_c2/run_kernel_stats.csv')):
    print('c2', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
echo r05k all done
