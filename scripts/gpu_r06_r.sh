#!/bin/bash
# Round-6 session R: same-box repeatability of the C2 line (three runs of the driver's form, one process each).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06r
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $O/c2_$i.log 2>&1
  rc=$?; echo "c2_$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
grep -h '^{' $O/c2_*.log | python3 -c "import json,sys; [print(round(json.loads(l)['value']/1e9,4), round(json.loads(l)['ms_per_step']*1e3,1)) for l in sys.stdin]"
echo r06r done
