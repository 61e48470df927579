#!/bin/bash
# Round 4, session C: the native executor with two batches planned ahead (tests, host cost at W = 8), the
# TranSparse forward with the operands split once (ts_fwd_x3s_kernel): its tests, the C6 line, a same-box
# A/B against ts_fwd_x3_kernel (KGE_TS_X3S=0) and one SQ counter pass; then the whole GPU suite.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 40 "$O/$n.log"; exit $rc; fi
}
run pytest_new 600 python3 -u -m pytest tests/test_native_exec_gpu.py tests/test_rccl_gpu.py tests/test_transparse_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
tail -n 2 $O/pytest_new.log
run host_probe 300 python3 scripts/shard_host_probe.py 8 20
grep '^{' $O/host_probe.log
run bench_c6 300 python3 bench.py --workload c6 --no-cpu-baseline
grep '^{' $O/bench_c6.log | cut -c1-600
AB="--workload c6 --steps 30 --warmup 5 --train-steps 0 --no-cpu-baseline"
run prof_c6 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c6 -o run -- python3 bench.py $AB
run prof_c6_old 300 env KGE_TS_X3S=0 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c6_old -o run -- python3 bench.py $AB
run pmc_c6_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    --kernel-trace --output-format csv -d $O/pmc_c6_sq -o run -- python3 bench.py --workload c6 --steps 10 --warmup 2 --train-steps 0 --no-cpu-baseline
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_gpu.log
echo r04c done
