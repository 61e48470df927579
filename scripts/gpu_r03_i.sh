#!/bin/bash
# Round-3 session I: A/B of the phased XCD-sliced order (KGE_XCD_PHASES) on the C2 headline and C4 step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/i
mkdir -p $O
for i in 1 2; do
  for ph in ${PHASES:-1 2 3 4}; do
    for wl in ${WLS:-c2 c4}; do
      KGE_XCD_PHASES=$ph timeout -k 10 300 python3 bench.py --workload $wl --steps 50 --no-cpu-baseline --train-steps 0 \
          --sharded-steps 0 > $O/${wl}_p${ph}_$i.json 2> $O/${wl}_p${ph}_$i.err || { tail -5 $O/${wl}_p${ph}_$i.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/${wl}_p${ph}_$i.json').read().strip().split(chr(10))[-1]); r=d['roofline']
print('$wl phases $ph run $i', 'value', round(d['value']/1e9,4), 'ms', round(d['ms_per_step'],4), 'kernel_us', round(r.get('kernel_avg_us',0),1))"
    done
  done
done
echo session-i done
