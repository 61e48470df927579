#!/bin/bash
# Round-3 session B: GPU tests, two-process exchange, default bench on the main build; then the TranSparse
# forward A/B (256-row 16-wave kernel = main, the 128-row kernel = KGE_TS_BIG=0, the 8-wave 256-row kernel =
# abtmp/ts) with its GPU tests and a kernel-trace profile of each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
STEPS=smoke,test,two,bench bash scripts/gpu_check.sh || exit $?
OUT=gpurun_out/ts_ab
mkdir -p $OUT
KGE_HIP_LIB=$R/abtmp/ts/libkge_hip.so timeout -k 10 300 python3 -u -m pytest tests/test_transparse_gpu.py -m gpu -q -x \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_ts8.log 2>&1
echo "tests ts8 rc=$?: $(tail -n 1 $OUT/tests_ts8.log)"
BA="--workload c6 --no-cpu-baseline --steps 20 --train-steps 5"
for i in 1 2; do
  for v in main old ts8; do
    case $v in
      main) env=""; lib=customknowledgegraphembedding_amd/libkge_hip.so ;;
      old) env="KGE_TS_BIG=0"; lib=customknowledgegraphembedding_amd/libkge_hip.so ;;
      ts8) env=""; lib=abtmp/ts/libkge_hip.so ;;
    esac
    env $env KGE_HIP_LIB=$R/$lib timeout -k 10 300 python3 bench.py $BA > $OUT/$v$i.json 2> $OUT/$v$i.err || exit $?
    python3 -c "
import json; d=json.load(open('$OUT/$v$i.json')); r=d['roofline']
print('$v$i', 'kernel_us', round(r['kernel_avg_us'],1), 'fp32eq_TF', round(r['fp32_equivalent_tflops'],1), 'frac_bf16', round(r['frac'],3), 'train_ms', round((d.get('train_step') or {}).get('ms_per_step',0),3))"
  done
done
echo session-b done
VARIANTS="main=customknowledgegraphembedding_amd/libkge_hip.so d1w3=abtmp/d1w3/libkge_hip.so" \
  TESTS="tests/test_train_gpu.py" bash scripts/ab_lib.sh || exit $?
echo session-b2 done
