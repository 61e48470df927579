#!/bin/bash
# Builds a variant of libkge_hip.so with extra compile flags into abtmp/<name>/ for same-box A/B runs
# (select it with KGE_HIP_LIB=abtmp/<name>/libkge_hip.so). Objects of translation units the flags do not
# touch can be taken from the main build by listing only the changed sources in SRCS.
# Usage: bash scripts/ab_build.sh <name> "<flags>" [sources...]
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
FLAGS=$2
shift 2
PKG=$R/customknowledgegraphembedding_amd
OUT=$R/abtmp/$NAME
mkdir -p "$OUT"
SRCS=${*:-$(ls $PKG/csrc/*.hip)}
pids=()
for s in $SRCS; do
  b=$(basename "$s" .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -ffp-contract=on \
      -I"$R/include" $FLAGS -c -o "$OUT/$b.o" "$s" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
objs=()
for o in $PKG/build/*.o; do
  b=$(basename "$o")
  if [ -f "$OUT/$b" ]; then objs+=("$OUT/$b"); else objs+=("$o"); fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libkge_hip.so" "${objs[@]}"
echo "$OUT/libkge_hip.so"
