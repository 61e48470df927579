#!/bin/bash
# Round 4, session F: the one-launch step (kge_step_forward_ws: row reductions in each row group's last slice
# block) - its tests, a same-box A/B against the two-launch step (KGE_STEP_FOLD=0) on C2 / C3 / C4, a kernel
# trace of the C2 bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 40 "$O/$n.log"; exit $rc; fi
}
run pytest_tile 600 python3 -u -m pytest tests/test_tile_gpu.py tests/test_configs_gpu.py tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_tile.log
AB="--steps 200 --warmup 20 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
for w in c2 c3 c4; do
  run ${w}_fold 300 python3 bench.py --workload $w $AB
  run ${w}_nofold 300 env KGE_STEP_FOLD=0 python3 bench.py --workload $w $AB
  run ${w}_fold2 300 python3 bench.py --workload $w $AB
  for f in ${w}_fold ${w}_nofold ${w}_fold2; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', 'G/s %.4f' % (d['value']/1e9), 'us/step %.1f' % (d['ms_per_step']*1e3))"; done
done
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_gpu.log
echo r04f done
