#!/bin/bash
# Round-3 session A: GPU tests + two-process exchange + bench on the main build, then the A/B of the fused
# train forward (abtmp/fast: gradient weights on hardware exp/log/rcp, packed InterHT Jacobian sums).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
STEPS=test,two,bench bash scripts/gpu_check.sh || exit $?
VARIANTS="main=customknowledgegraphembedding_amd/libkge_hip.so fast=abtmp/fast/libkge_hip.so" \
  TESTS="tests/test_train_gpu.py" bash scripts/ab_lib.sh || exit $?
echo session-a done
