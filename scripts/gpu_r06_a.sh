#!/bin/bash
# Round-6 first session: the GPU suite, the headline bench line and its kernel trace on this round's tree.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06a
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi  # 1: test failures (go on); anything else: stop
}
run new 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_train_c2_gpu.py tests/test_trained_range_gpu.py tests/test_planned_gpu.py tests/test_eval_gpu.py -k 'c2 or d1000 or separated or row_order or caller or without_entity or rotate or b_direct'
run c5 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_configs_gpu.py -k c5
run tsprobe_old 600 env KGE_HIP_LIB=$R/abtmp/libkge_pre_ts_rule.so python3 scripts/ts_many_rel_probe.py
run tsprobe 600 python3 scripts/ts_many_rel_probe.py
run sweep 600 python3 scripts/sweep_probe.py
run gemm 600 python3 scripts/gemm_form_probe.py
run scaling 600 python3 scripts/shard_scaling_probe.py
run tests 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run bench_c2 600 python3 bench.py
run prof_c2 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --sharded-steps 0
tail -n 2 $O/bench_c2.log
echo r06a done
