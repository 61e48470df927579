#!/bin/bash
# round 5: tile forms (rows per group 16/12/8, waves per block 8/12/16) on the unplanned step, C2 C3 C4
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05y
mkdir -p $O
for wl in c2 c3 c4; do
  timeout -k 10 200 python3 -u scripts/tile_forms_probe.py $wl >> $O/forms.json 2>> $O/forms.err || { tail -20 $O/forms.err; exit 1; }
done
cat $O/forms.json
