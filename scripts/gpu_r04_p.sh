#!/bin/bash
# Round 4: (1) tile kernel with the query build after the scatter and the first gather in flight under it
# (abtmp/pre) vs the shipped order (the in-tree library): parity (tile / config / parity tests incl. the every-row full-size checks)
# and C2 / C3 / C4 kernel traces, alternating; (2) TranSparse grouped kernel 3-deep prefetch (abtmp/xg3);
# (3) the row-sharded host cost as the C2 line now reports it (per-call median).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
PRE=$R/abtmp/pre/libkge_hip.so
XG3=$R/abtmp/xg3/libkge_hip.so
run pytest_pre 600 env KGE_HIP_LIB=$PRE python3 -u -m pytest tests/test_tile_gpu.py tests/test_configs_gpu.py tests/test_parity_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_pre.log
run pytest_xg3 600 env KGE_HIP_LIB=$XG3 python3 -u -m pytest tests/test_transparse_gpu.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_xg3.log
for w in c2 c3 c4; do
  AB="--workload $w --steps 100 --warmup 10 --train-steps 0 --sharded-steps 0 --no-cpu-baseline"
  for v in base pre base2 pre2; do
    if [ "${v#pre}" != "$v" ]; then L="env KGE_HIP_LIB=$PRE"; else L=""; fi
    run ${w}_$v 300 $L rocprofv3 --kernel-trace --stats --output-format csv -d $O/${w}_$v -o run -- python3 bench.py $AB
  done
done
AB="--workload c6 --steps 50 --warmup 5 --train-steps 0 --no-cpu-baseline"
for v in base xg3 base2 xg32; do
  if [ "${v#xg3}" != "$v" ]; then L="env KGE_HIP_LIB=$XG3"; else L=""; fi
  run c6_$v 300 $L rocprofv3 --kernel-trace --stats --output-format csv -d $O/c6_$v -o run -- python3 bench.py $AB
done
run hostcost 600 python3 bench.py --no-cpu-baseline --train-steps 0 --steps 5 --warmup 1
grep -h '^{' $O/hostcost.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.readline()); h=d['yago3_10_shard_sim8']['host_us_per_rank_step']
print('hostcost', round(h['python_path']['total'],1), h['native'])"
echo r04p done
