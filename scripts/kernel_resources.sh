#!/bin/bash
# Per-kernel VGPR/SGPR/LDS/scratch of the built gfx950 code objects (build/*.o).
# Usage: bash scripts/kernel_resources.sh [pattern]
cd "$(dirname "$0")/.." || exit 1
LLVM=/opt/rocm/lib/llvm/bin
tmp=$(mktemp -d)
for o in ${BUILD_DIR:-rag-cobweb_amd/build}/*.o; do
  $LLVM/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fb.bin "$o" 2>/dev/null || continue
  $LLVM/clang-offload-bundler --unbundle --type=o --input=$tmp/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --output=$tmp/k.co 2>/dev/null || continue
  $LLVM/llvm-readelf --notes $tmp/k.co | grep -E "^\s+(- )?\.(name|private_segment_fixed_size|vgpr_count|sgpr_count|group_segment_fixed_size|vgpr_spill_count|agpr_count):" |
    paste - - - - - - - | awk -v f="$(basename "$o")" '{printf "%-14s agpr=%-4s lds=%-7s scratch=%-5s sgpr=%-4s vgpr=%-4s spill=%-3s %s\n", f, $3, $5, $9, $11, $13, $15, substr($7,1,90)}'
done | grep -E "${1:-.}"
rm -rf "$tmp"
