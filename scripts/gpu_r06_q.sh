#!/bin/bash
# Round-6 session Q: the plane GEMM on 16 x 16 x 32 MFMAs (form 5) against the 32 x 32 x 16 forms at C5's shape.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 scripts/gemm_form_probe.py > $O/gemm.log 2>&1; rc=$?
echo "gemm rc=$rc"; grep '^{' $O/gemm.log || tail -20 $O/gemm.log
echo r06q done
