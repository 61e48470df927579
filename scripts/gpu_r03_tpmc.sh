#!/bin/bash
# PMC of the step orders at C2 (tile vs xcd) and of the locality probe: FETCH_SIZE and L2 hit/miss passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
O=$R/gpurun_out/tpmc
mkdir -p $O
for o in ${ORDERS:-tile xcd}; do
  i=0
  for C in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    i=$((i+1))
    KGE_STEP_ORDER=$o timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$o/p$i -o run -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --sharded-steps 0 --train-steps 0 > $O/$o.p$i.log 2>&1
    rc=$?; echo "$o pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$o.p$i.log; exit $rc; }
  done
done
if [ -n "${PROBE:-}" ]; then
  i=0
  for C in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/probe/p$i -o run -- ./tools/locality_probe > $O/probe.p$i.log 2>&1
    rc=$?; echo "probe pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
fi
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("O_DIR", "gpurun_out/tpmc")
for f in sorted(glob.glob(O + "/*/p*/run_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        if "tile" in k or "xcd" in k or "neg_rows" in k or "gather" in k or "pairs" in k:
            print(f.split("/")[-3], f.split("/")[-2], k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in d.items()}, "n", len(next(iter(d.values()))))
PY
echo tpmc done
