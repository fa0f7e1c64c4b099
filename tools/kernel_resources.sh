#!/bin/bash
# Per-kernel VGPR / SGPR / scratch / spill counts of the gfx950 code object inside flink_amd/libflink_amd.so.
# usage: tools/kernel_resources.sh [kernel-name-regexp]
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section .hip_fatbin=$T/fat.bin "$(dirname "$0")/../flink_amd/libflink_amd.so" $T/x.so
$B/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/co.o
$B/llvm-readelf --notes $T/co.o | grep -E "^ +\.name:|private_segment_fixed_size|\.vgpr_count|vgpr_spill|sgpr_spill" |
  awk -v re="${1:-.}" '/\.name:/{show = ($2 ~ re)} show'
rm -rf $T
