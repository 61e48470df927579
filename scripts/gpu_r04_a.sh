#!/bin/bash
# Round 4, first GPU session: GPU tests (incl. RCCL at world 1), host cost of the row-sharded step, C2/C3
# bench lines and kernel traces, and one VALU counter pass on the C3 tile kernel after the hardware sqrt.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
run pytest_rccl 300 python3 -u -m pytest tests/test_rccl_gpu.py -v -x -p no:cacheprovider --timeout 120 --timeout-method thread
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_gpu.log
run host_probe 300 python3 scripts/shard_host_probe.py 8 20
head -n 1 $O/host_probe.log
run bench_c2 600 python3 bench.py --sharded-steps 0 --no-cpu-baseline
run bench_c3 600 python3 bench.py --workload c3 --no-cpu-baseline
run prof_c3 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --workload c3 --steps 50 --warmup 5 --no-cpu-baseline --train-steps 0
run pmc_c3_valu 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    --kernel-trace --output-format csv -d $O/pmc_c3_valu -o run -- \
    python3 bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --train-steps 0
# tile A/B (InterHT C2): relation third staged per item (base) vs read from LDS in the score (q2lds), 12 / 16 waves
run pytest_q2 600 env KGE_HIP_LIB=$R/abtmp/q2lds/libkge_hip.so KGE_TILE_WAVES=16 python3 -u -m pytest tests/test_tile_gpu.py tests/test_configs_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_q2.log
AB="--steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
run ab_base 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ab_base -o run -- python3 bench.py $AB
run ab_q2 300 env KGE_HIP_LIB=$R/abtmp/q2lds/libkge_hip.so rocprofv3 --kernel-trace --stats --output-format csv -d $O/ab_q2 -o run -- python3 bench.py $AB
run ab_q2w16 300 env KGE_HIP_LIB=$R/abtmp/q2lds/libkge_hip.so KGE_TILE_WAVES=16 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ab_q2w16 -o run -- python3 bench.py $AB
run ab_base2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ab_base2 -o run -- python3 bench.py $AB
echo r04a done
