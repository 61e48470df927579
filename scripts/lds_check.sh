#!/bin/bash
# C5 eval GEMM + c6 TranSparse: parity tests, bench lines, one LDS-counter pass each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/lds
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_eval_gpu.py tests/test_transparse_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/lds/tests.log 2>&1 || { echo tests rc=$?; tail -20 gpurun_out/lds/tests.log; exit 1; }
tail -1 gpurun_out/lds/tests.log
for W in c5 c6; do
  timeout -k 10 200 python3 bench.py --workload $W --steps 20 --train-steps 0 > gpurun_out/lds/$W.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['roofline']['achieved'], d['roofline']['frac'])" gpurun_out/lds/$W.json
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL --kernel-trace --output-format csv -d "$R/gpurun_out/lds/pmc_$W" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --train-steps 0 --sharded-steps 0 --workload $W > gpurun_out/lds/pmc_$W.log 2>&1 || exit $?
done
echo done
