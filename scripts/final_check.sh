#!/bin/bash
# Round-end evidence on one GPU box: smoke, GPU tests, default bench, kernel-trace stats, PMC passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
STEPS=smoke,test,bench,prof bash scripts/gpu_check.sh || exit $?
bash scripts/pmc.sh ${1:-c2} || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc/${1:-c2} gpurun_out/pmc_${1:-c2}.json > gpurun_out/pmc_${1:-c2}.txt
echo final done
