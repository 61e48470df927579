#!/bin/bash
# Tile-kernel A/B by environment knobs: kernel-trace average of the step kernels per (workload, knobs).
# CASES="c2: c2:KGE_TILE_DRY=1 ..." (workload:VAR=VAL,VAR=VAL)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
O=$R/gpurun_out/tab
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -n 1 $O/tests.log)"; [ $rc -ne 0 ] && { tail -30 $O/tests.log; exit $rc; }
fi
i=0
for c in $CASES; do
  i=$((i+1))
  wl=${c%%:*}; kv=${c#*:}
  envs=$(echo "$kv" | tr ',' ' ')
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$i -o run -- \
      python3 bench.py --workload $wl --steps 30 --warmup 3 --no-cpu-baseline --train-steps 0 --sharded-steps 0 > $O/c$i.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "case $c rc=$rc"; tail -5 $O/c$i.log; exit $rc; }
  python3 - "$c" "$O/c$i/run_kernel_stats.csv" "$O/c$i.log" <<'PY'
import csv, json, sys
c, f, log = sys.argv[1:]
try:
    d = json.loads(open(log).read().strip().splitlines()[-1]); v = "%.4f G/s %.1f us" % (d["value"] / 1e9, d["ms_per_step"] * 1e3)
except Exception as e:
    v = "?"
ks = []
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "tile" in n or "xcd" in n or "neg_rows" in n or "step_fwd" in n:
        ks.append("%s<%s> %.1f" % (n.split("(")[0].split("::")[-1][:22], n[n.find("<") + 1:n.find(">")], float(r["AverageNs"]) / 1e3))
print(c, "|", v, "|", "; ".join(ks))
PY
done
echo tab done
