#!/bin/bash
# Register / spill report of ONE kernel instantiation (device-only compile, seconds): for A/B of register use.
# Usage: bash scripts/kreg.sh '<explicit instantiation>' [extra hipcc flags]
#   e.g. bash scripts/kreg.sh 'template __global__ void step_fwd_grad_kernel<4, false, 4, 4, 2>(ScoreParams);' -DKGE_FG_WPE=3
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
printf '#include "kge_device.h"\nnamespace kge_impl {\n%s\n}\n' "$1" > "$T/k.hip"
shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-result -ffp-contract=on -I"$R/include" \
    -I"$R/customknowledgegraphembedding_amd/csrc" --cuda-device-only "$@" -c -o "$T/k.o" "$T/k.hip"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/k.o" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/k.co"
/opt/rocm/lib/llvm/bin/llvm-readelf -n "$T/k.co" | grep -E "\.name:|vgpr_count|vgpr_spill|private_segment_fixed"
rm -rf "$T"
