#!/bin/bash
# MFMA / LDS counter passes over one workload (one group per pass): busy cycles, LDS conflicts.
# Usage: bash scripts/pmc_mfma.sh <workload>   -> gpurun_out/pmc_mfma/<workload>/p*/
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=${1:-c5}
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/pmc_mfma/$W"
i=0
for CTRS in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" \
            "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_MFMA SQ_WAVES" "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES" \
            "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  echo "== pass $i: $CTRS"
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_mfma/$W/p$i" -o run -- \
      python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --train-steps 2 --sharded-steps 0 --workload "$W" \
      > "$R/gpurun_out/pmc_mfma/$W/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc: stopping"; exit $rc; fi
done
echo done
