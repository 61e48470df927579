#!/bin/bash
# round 5: the planner handle (9-argument step call, double-buffered outputs); C2 bench as the driver runs it
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_planned_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $O/bench_c2_20_$k.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2_20_$k.json')); r=d['roofline']; print(d['ms_per_step'], r['host_us_per_step_median'], r['event_group_step_us'], r['step_us_head_batch'], r['step_us_tail_batch'], r['unplanned_step_us'])"
done
KGE_BENCH_UNPLANNED=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $O/bench_c2_unplanned.json 2>> $O/bench_c2.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_c2_unplanned.json')); r=d['roofline']; print('unplanned', d['ms_per_step'], r['host_us_per_step_median'], r['event_group_step_us'])"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 10 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $O/bench_c2_200.json 2>> $O/bench_c2.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_c2_200.json')); r=d['roofline']; print('200', d['ms_per_step'], r['host_us_per_step_median'], r['step_us_head_batch'], r['step_us_tail_batch'])"
