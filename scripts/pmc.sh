#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, --kernel-trace only beside --pmc).
# Usage: bash scripts/pmc.sh [workload]   -> gpurun_out/pmc/<pass>/...counter_collection.csv
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=${1:-c2}
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/pmc/$W"
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
            "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
            "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "== pass $i: $CTRS"
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/$W/p$i" -o run -- \
      python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --sharded-steps 0 --train-steps 5 --workload "$W" > "$R/gpurun_out/pmc/$W/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc: stopping"; exit $rc; fi
done
echo done
