#!/bin/bash
# round 5: PMC of the shipped plane GEMM (MFMA-interleaved stores and loads; query rows written as planes) at C5
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
export TMPDIR=/tmp
P=gpurun_out/pmc/c5f
mkdir -p $P
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$R/$P/p$i" -o run -- \
      python3 "$R/bench.py" --workload c5 --steps 5 --warmup 2 > "$R/$P/p$i.log" 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
cd "$R" && python3 scripts/pmc_summary.py $P $P/summary.json > $P/summary.txt && grep -A20 "gemm_nt_x3p" $P/summary.txt
