#!/bin/bash
# Round-3 session J: GPU tests; C3 (RotatE query build without spills) and C4 with KGE_XCD_DEPTH 1 / 2.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/j
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in c3:1 c4:1 c4:2; do
    wl=${v%%:*}; dp=${v##*:}
    KGE_XCD_DEPTH=$dp timeout -k 10 300 python3 bench.py --workload $wl --steps 50 --no-cpu-baseline --train-steps 0 \
        --sharded-steps 0 > $O/${wl}_d${dp}_$i.json 2> $O/${wl}_d${dp}_$i.err || { tail -5 $O/${wl}_d${dp}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${wl}_d${dp}_$i.json').read().strip().split(chr(10))[-1]); r=d['roofline']
print('$wl depth $dp run $i', 'value', round(d['value']/1e9,4), 'ms', round(d['ms_per_step'],4), 'kernel_us', round(r.get('kernel_avg_us',0),1))"
  done
done
echo session-j done
