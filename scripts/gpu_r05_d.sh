#!/bin/bash
# round 5: PMC of the C5 eval GEMM (gemm_nt_x3s_kernel): MFMA busy, waits, LDS conflicts, co-issue; two passes
set -o pipefail
cd "$(dirname "$0")/.."
R=$(pwd)
O=gpurun_out/pmc/c5
mkdir -p $O
export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$R/$O/p$i" -o run -- \
      python3 "$R/bench.py" --workload c5 --steps 5 --warmup 2 > "$R/$O/p$i.log" 2>&1 || { echo "pass $i rc=$?"; tail -5 "$R/$O/p$i.log"; exit 1; }
done
cd "$R" && python3 scripts/pmc_summary.py $O $O/summary.json > $O/summary.txt && grep -A20 "gemm_nt_x3s" $O/summary.txt
