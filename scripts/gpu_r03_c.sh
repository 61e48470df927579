#!/bin/bash
# Round-3 session C: rank 0's kernels of the 8-rank row-sharded forward (scripts/shard_probe.py), default
# candidate order and KGE_STEP_ORDER=row, then a kernel-trace profile of the default order.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/probe
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/shard_probe.py --chunks 1,2,4 > $OUT/default.log 2>&1 || { tail -20 $OUT/default.log; exit 1; }
tail -n 1 $OUT/default.log
KGE_STEP_ORDER=row timeout -k 10 300 python3 -u scripts/shard_probe.py --chunks 1,2,4 > $OUT/row.log 2>&1 || { tail -20 $OUT/row.log; exit 1; }
tail -n 1 $OUT/row.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o probe -- python3 scripts/shard_probe.py --chunks 4 --reps 5 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -n 1)
cut -d, -f1-8 "$f" | head -n 30
echo session-c done
