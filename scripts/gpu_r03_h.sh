#!/bin/bash
# Round-3 session H: PMC passes (scripts/pmc.sh) for the workloads given as arguments, summarised into
# gpurun_out/pmc/pmc_<w>.json (source hash of the library they ran).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for W in "$@"; do
  bash scripts/pmc.sh "$W" || exit $?
  python3 scripts/pmc_summary.py "gpurun_out/pmc/$W" "gpurun_out/pmc/pmc_$W.json" > "gpurun_out/pmc/$W/summary.txt" 2>&1 || exit 1
  echo "$W summarised"
done
echo session-h done
