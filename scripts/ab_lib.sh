#!/bin/bash
# Same-box A/B of library builds (scripts/ab_build.sh): GPU tests under each variant (TESTS), alternating
# bench runs (BENCH_ARGS) printing the step and train-step times, then a kernel-trace profile of each.
# Usage: VARIANTS="main=customknowledgegraphembedding_amd/libkge_hip.so x=abtmp/x/libkge_hip.so" bash scripts/ab_lib.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/ab_lib
mkdir -p $OUT
BENCH_ARGS=${BENCH_ARGS:---workload c2 --no-cpu-baseline --sharded-steps 0 --steps 20 --train-steps 50}
for v in $VARIANTS; do
  n=${v%%=*}; lib=${v#*=}
  if [ -n "${TESTS:-}" ]; then
    KGE_HIP_LIB=$R/$lib timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -q -x -p no:cacheprovider --timeout 300 \
        --timeout-method thread > $OUT/tests_$n.log 2>&1
    rc=$?; echo "tests $n rc=$rc: $(tail -n 1 $OUT/tests_$n.log)"; [ $rc -ne 0 ] && exit $rc
  fi
done
for i in 1 2; do
  for v in $VARIANTS; do
    n=${v%%=*}; lib=${v#*=}
    KGE_HIP_LIB=$R/$lib timeout -k 10 300 python3 bench.py $BENCH_ARGS > $OUT/$n$i.json 2> $OUT/$n$i.err || exit $?
    python3 -c "
import json; d=json.load(open('$OUT/$n$i.json')); t=d.get('train_step') or {}
print('$n$i', 'value', round(d['value']/1e9,4), 'step_us', round(d['ms_per_step']*1e3,1), 'train_ms', round(t.get('ms_per_step',0),4))"
  done
done
export TMPDIR=/tmp
for v in $VARIANTS; do
  n=${v%%=*}; lib=${v#*=}
  KGE_HIP_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$n" -o run -- \
      python3 "$R/bench.py" $BENCH_ARGS > /dev/null 2>&1 || exit $?
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof_$n/run_kernel_stats.csv')):
    if 'kge' in r['Name'] or 'neg_rows' in r['Name']:
        print('$n', r['Name'][:75], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
done
echo ok
