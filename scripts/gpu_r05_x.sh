#!/bin/bash
# round 5 (profiling A/B, not shipped unless it wins): the tile sweep in KGE_SWEEP_PHASES phases per XCD slice
# (waves entering a phase wait, bounded, until 3/4 of the slice's waves have): planned-step tests under the
# variant, then device us per step (scripts/plan_probe.py planned_tail) for main / 8 / 16 phases, alternating
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05x
mkdir -p $O
KGE_HIP_LIB=$R/abtmp/ph8/libkge_hip.so timeout -k 10 400 python3 -u -m pytest tests/test_planned_gpu.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_ph8.log 2>&1 || { tail -30 $O/tests_ph8.log; exit 1; }
echo "tests ph8: $(tail -n 1 $O/tests_ph8.log)"
for i in 1 2; do
  for v in main=customknowledgegraphembedding_amd/libkge_hip.so ph8=abtmp/ph8/libkge_hip.so ph16=abtmp/ph16/libkge_hip.so; do
    n=${v%%=*}; lib=${v#*=}
    for wl in c2 c3 c4; do
      KGE_HIP_LIB=$R/$lib timeout -k 10 200 python3 -u scripts/plan_probe.py $wl > $O/probe_${n}_${wl}_$i.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/probe_${n}_${wl}_$i.json')); print('$n $wl $i', round(d['planned_tail'],1), round(d['unplanned'],1))"
    done
  done
done
echo r05x done
