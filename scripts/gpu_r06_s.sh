#!/bin/bash
# Round-6 session S: the C2 line with its planned / unplanned comparison interleaved (bench.py's plan_ab), twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06s
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 env KGE_PMC_DIR=gpurun_out/pmc python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $O/c2_$i.log 2>&1
  rc=$?; echo "c2_$i rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/c2_$i.log; exit $rc; }
done
grep -h '^{' $O/c2_*.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']
    print(round(d['value']/1e9,4), round(d['ms_per_step']*1e3,1), round(r['kernel_avg_us'],1), round(r['planned_step_us'],1), round(r['unplanned_step_us'],1))"
echo r06s done
