#!/bin/bash
# Round 4, session G: the eval GEMM with the operands split once (gemm_nt_x3s_kernel): its tests, the C5 line
# and a same-box kernel-trace A/B against gemm_nt_f32x3_kernel (KGE_GEMM_X3S=0); then the whole GPU suite.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 40 "$O/$n.log"; exit $rc; fi
}
run pytest_eval 600 python3 -u -m pytest tests/test_eval_gpu.py tests/test_configs_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_eval.log
run bench_c5 300 python3 bench.py --workload c5 --no-cpu-baseline
grep '^{' $O/bench_c5.log | cut -c1-300
AB="--workload c5 --steps 30 --warmup 5 --no-cpu-baseline"
run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py $AB
run prof_c5_old 300 env KGE_GEMM_X3S=0 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_old -o run -- python3 bench.py $AB
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_gpu.log
echo r04g done
