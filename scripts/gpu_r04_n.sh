#!/bin/bash
# Round 4: the row-sharded host cost as bench.py's C2 line reports it, with and without the work before it
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04n
mkdir -p $O
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
show() { grep -h '^{' $O/$1.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.readline()); h=d['yago3_10_shard_sim8']['host_us_per_rank_step']
print('$1', round(h['python_path']['total'],1), round(h['native']['step_us'],1), round(h['native']['step_us_mean'],1), round(h['native']['blocked_us_per_step'],1), round(h['native']['wall_us_per_step'],1))"; }
run default 600 python3 bench.py --no-cpu-baseline
show default
run notrain 600 python3 bench.py --no-cpu-baseline --train-steps 0
show notrain
run short 600 python3 bench.py --no-cpu-baseline --train-steps 0 --steps 5 --warmup 1
show short
run default2 600 python3 bench.py --no-cpu-baseline
show default2
echo r04n done
