#!/bin/bash
# round 5: the eval GEMM on pre-split planes (tests, C5 bench both forms, rocprof, PMC of the new kernel)
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_eval_gpu.py "tests/test_configs_gpu.py::test_c5_fb15k_filtered_ranks_full_entity_set" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
KGE_BENCH_EVAL_SPLIT=staging timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 5 > $O/bench_c5_staging.json 2>> $O/bench_c5.err || exit 1
python3 -c "
import json
for f in ('$O/bench_c5.json', '$O/bench_c5_staging.json'):
    d = json.load(open(f)); r = d['roofline']; print(f, d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c5 -o run -- python3 $R/bench.py --workload c5 --steps 20 --warmup 5 > $R/$O/prof_c5.log 2>&1 || exit 1
cd $R
P=gpurun_out/pmc/c5p
mkdir -p $P
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$R/$P/p$i" -o run -- \
      python3 "$R/bench.py" --workload c5 --steps 5 --warmup 2 > "$R/$P/p$i.log" 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
cd "$R" && python3 scripts/pmc_summary.py $P $P/summary.json > $P/summary.txt && grep -A20 "gemm_nt_x3p" $P/summary.txt
