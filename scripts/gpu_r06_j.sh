#!/bin/bash
# Round-6 session J: vendor GEMM on the six products concatenated along K (what hipBLASLt sustains at C5's shape).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 scripts/blaslt_probe.py > $O/blaslt.log 2>&1; rc=$?
echo "blaslt rc=$rc"; tail -5 $O/blaslt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/blaslt_probe.py > $O/prof.log 2>&1; echo "prof rc=$?"
echo r06j done
