#!/bin/bash
# A/B of kge_step_forward's candidate order (KGE_STEP_ORDER=row|xcd) on one GPU box: parity tests of the
# step forward under the XCD order, alternating C2 bench runs, then a kernel-trace profile of each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/ab_order
W=${WORKLOAD:-c2}
KGE_XCD_DEPTH=${TEST_DEPTH:-1} KGE_STEP_ORDER=xcd timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_parity_gpu.py tests/test_configs_gpu.py} -m gpu -q -x \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab_order/tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/ab_order/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for o in row xcd xcd1; do
    KGE_XCD_DEPTH=${o:3:1} KGE_STEP_ORDER=${o:0:3} timeout -k 10 300 python3 bench.py --workload $W --no-cpu-baseline --sharded-steps 0 --train-steps 0 \
        --steps 50 > gpurun_out/ab_order/$o$i.json 2> gpurun_out/ab_order/$o$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_order/$o$i.json')); r=d['roofline']; print('$o$i', round(d['value']/1e9,4), 'G/s', round(d['ms_per_step']*1e3,1), 'us/step', round(r['kernel_avg_us'],1), 'us kernels')"
  done
done
export TMPDIR=/tmp
for o in row xcd xcd1; do
  KGE_XCD_DEPTH=${o:3:1} KGE_STEP_ORDER=${o:0:3} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ab_order/prof_$o" -o run -- \
      python3 "$R/bench.py" --workload $W --no-cpu-baseline --sharded-steps 0 --train-steps 0 --steps 50 > /dev/null 2>&1 || exit $?
done
echo ok
