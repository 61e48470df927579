#!/bin/bash
# Round-3 tile session: parity of the row-group x XCD-slice tile form, then same-box A/B of the step orders
# (c2 c3 c4 kernel time in the bench line), then the locality probe. Each GPU step has its own limit and a
# failing step ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/tile
mkdir -p $O
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
run pytest_tile 600 python3 -u -m pytest tests/test_tile_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 2 $O/pytest_tile.log
for wl in ${WLS:-c2 c3 c4}; do
  for o in tile xcd; do
    KGE_STEP_ORDER=$o run bench_${wl}_$o 300 python3 bench.py --workload $wl --no-cpu-baseline --train-steps 0 --sharded-steps 0
    python3 -c "import json,sys; d=json.loads(open('$O/bench_${wl}_$o.log').read().strip().splitlines()[-1]); print('$wl $o', round(d['value']/1e9,4), 'G/s', d['ms_per_step'], 'ms', d.get('roofline',{}).get('frac'))"
  done
done
run probe 120 ./tools/locality_probe
cat $O/probe.log
echo tile done
