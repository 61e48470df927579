#!/bin/bash
# Round 4, session D: TranSparse single/tail-batch rows with all columns per block (ts_fwd_x3g_kernel) - tests,
# the C6 line and a kernel trace; the native executor's device timeline at W = 8 (K = 2 and 1); the C2 headline
# with consecutive steps on two streams (A/B, --streams 2) against one.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 40 "$O/$n.log"; exit $rc; fi
}
run pytest_ts 600 python3 -u -m pytest tests/test_transparse_gpu.py tests/test_native_exec_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
tail -n 2 $O/pytest_ts.log
run prof_c6 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c6 -o run -- python3 bench.py --workload c6 --steps 30 --warmup 5 --train-steps 0 --no-cpu-baseline
grep '^{' $O/prof_c6.log | cut -c1-400
run tl_k2 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_k2 -o run -- python3 scripts/native_timeline.py 2 40
python3 scripts/native_timeline.py --analyze $O/tl_k2 > $O/tl_k2.json; cat $O/tl_k2.json
run tl_k1 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_k1 -o run -- python3 scripts/native_timeline.py 1 40
python3 scripts/native_timeline.py --analyze $O/tl_k1 > $O/tl_k1.json; cat $O/tl_k1.json
run c2_s1 300 python3 bench.py --steps 200 --warmup 20 --train-steps 0 --sharded-steps 0 --no-cpu-baseline
run c2_s2 300 python3 bench.py --steps 200 --warmup 20 --train-steps 0 --sharded-steps 0 --no-cpu-baseline --streams 2
run c2_s1b 300 python3 bench.py --steps 200 --warmup 20 --train-steps 0 --sharded-steps 0 --no-cpu-baseline
for f in c2_s1 c2_s2 c2_s1b; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value']/1e9, d['ms_per_step']*1e3)"; done
run c3_s1 300 python3 bench.py --workload c3 --steps 200 --warmup 20 --train-steps 0 --no-cpu-baseline
run c3_s2 300 python3 bench.py --workload c3 --steps 200 --warmup 20 --train-steps 0 --no-cpu-baseline --streams 2
for f in c3_s1 c3_s2; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value']/1e9, d['ms_per_step']*1e3)"; done
echo r04d done
