#!/bin/bash
# Round 4: pRotatE's per-element sin on the hardware unit (abtmp/prothw): the whole GPU suite on it, then the
# pRotatE step time (scripts/protate_probe.py) against the shipped library, alternating.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r04v
mkdir -p $O
export TMPDIR=/tmp
run() {  # name limit cmd...
  local n=$1 l=$2; shift 2
  timeout -k 10 "$l" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 30 "$O/$n.log"; exit $rc; fi
}
F=$R/abtmp/prothw/libkge_hip.so
run pytest_prothw 900 env KGE_HIP_LIB=$F python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread
tail -n 1 $O/pytest_prothw.log
for v in base hw base2 hw2; do
  L=""
  case $v in hw*) L="env KGE_HIP_LIB=$F";; esac
  run p_$v 300 $L python3 scripts/protate_probe.py
  echo "$v $(grep '^{' $O/p_$v.log)"
done
echo r04v done
