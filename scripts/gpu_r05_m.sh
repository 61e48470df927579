#!/bin/bash
# round 5: the tile sweep's candidate loads under branches (cond, the round-4 form) vs unconditional (uncond), same
# box, alternating: C2 / C3 / C4 step device time (plan_probe planned_tail) and kernel trace at C2
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for n in cond uncond; do
    for wl in c2 c3 c4; do
      KGE_HIP_LIB=$R/abtmp/$n/libkge_hip.so timeout -k 10 200 python3 -u scripts/plan_probe.py $wl > $O/probe_${n}_${wl}_$i.json 2>> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/probe_${n}_${wl}_$i.json')); print('$n $wl $i', round(d['planned_tail'],1), round(d['unplanned'],1))"
    done
  done
done
echo r05m done
