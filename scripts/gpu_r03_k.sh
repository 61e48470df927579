#!/bin/bash
# Round-3 session K: GPU tests; C3 and C2 lines with train steps (RotatE query build in chunks of 4,
# RotatE Jacobian on rsq), C3 kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for wl in c3 c2; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 50 --no-cpu-baseline --sharded-steps 0 --train-steps 30 \
      > $O/$wl.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$wl.json').read().strip().split(chr(10))[-1]); r=d['roofline']; t=d.get('train_step') or {}
print('$wl', 'value', round(d['value']/1e9,4), 'ms', round(d['ms_per_step'],4), 'kernel_us', round(r.get('kernel_avg_us',0),1), 'frac', r.get('frac'), 'train_ms', t.get('ms_per_step'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --workload c3 --steps 30 --no-cpu-baseline --sharded-steps 0 --train-steps 20 > /dev/null 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_c3/run_kernel_stats.csv')):
    print(r['Name'][:75], r['Calls'], round(float(r['AverageNs'])/1e3, 1))" | head -12
echo session-k done
