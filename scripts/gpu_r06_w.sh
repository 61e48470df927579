#!/bin/bash
# Round-6 session W: the driver's short C2 form with the memory-side pre-warm (bench.py device_prewarm) against
# KGE_BENCH_PREWARM=0, alternating, three each; then C3 and C4 once each way.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06w
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for pw in 1 0; do
    timeout -k 10 300 env KGE_BENCH_PREWARM=$pw python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $O/c2_pw${pw}_$i.log 2>&1
    rc=$?; echo "c2 pw=$pw #$i rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/c2_pw${pw}_$i.log; exit $rc; }
  done
done
for W in c3 c4; do
  for pw in 1 0; do
    timeout -k 10 300 env KGE_BENCH_PREWARM=$pw python3 bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0 > $O/${W}_pw${pw}.log 2>&1
    rc=$?; echo "$W pw=$pw rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/${W}_pw${pw}.log; exit $rc; }
  done
done
for f in $O/*.log; do grep -h '^{' $f | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e9,4), round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_avg_us'],1), bool(d.get('device_prewarm')))"; done
echo r06w done
