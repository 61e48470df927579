#!/bin/bash
# Round 4, closing session on the shipped build (source hash unchanged since gpu_r04_final.sh, so the committed
# PMC summaries still pair with it): the whole GPU suite (now with the every-row full-size parity tests), smoke,
# and the C2 line again (its row-sharded host cost now the per-call median).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/final4b
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$O/$n.log"; exit $rc; fi
}
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_gpu.log
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
run bench_c2 600 python3 bench.py
echo final4b done
