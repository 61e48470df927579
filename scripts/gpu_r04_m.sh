#!/bin/bash
# Round 4: host cost of the row-sharded step, fresh process vs inside bench's sequence (scripts/host_cost_ab.py)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04m
mkdir -p $O
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
for v in fresh after_sim after_gc fresh after_sim after_gc; do
  run $v 300 python3 scripts/host_cost_ab.py $v
  grep '^{' $O/$v.log
done
echo r04m done
