#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a fault / abort / timeout (rc >= 124) ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
STEPS=${STEPS:-smoke,test,bench,prof}
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
[[ $STEPS == *smoke* ]] && step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *test* ]] && step pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
[[ $STEPS == *two* ]] && step shard_two_proc 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 scripts/shard_two_proc.py
[[ $STEPS == *bench* ]] && step bench 600 python3 bench.py
for wl in ${WORKLOADS:-}; do
  step "bench_$wl" 600 python3 bench.py --workload "$wl" ${BENCH_ARGS:-}
done
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
      python3 "$R/bench.py" --steps 50 --warmup 5 --no-cpu-baseline
fi
echo done
