#!/bin/bash
# Register / spill / LDS metadata of the gfx950 kernels in one object file:
#   bash tools/kernel_regs.sh conformer-nemo_amd/csrc/build/gemm.o [name-regex]
set -e
O=${1:?object}; P=${2:-.}
T=$(mktemp -d)
L=/opt/rocm/lib/llvm/bin
$L/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$O"
$L/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
$L/llvm-readelf --notes $T/k.co | grep -E "^ +\.group_segment_fixed_size|^ +\.name:|\.vgpr_count|\.vgpr_spill_count|\.agpr_count" \
  | paste - - - - - | sed 's/  */ /g' | grep -E "$P" || true
rm -rf $T
