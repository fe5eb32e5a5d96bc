#!/bin/bash
# VGPRs / scratch / spills of every kernel in a built libgmt.so (gfx950 code
# objects, AMDGPU metadata notes):  scripts/lib_resources.sh LIB [filter]
lib=$1; filt=${2:-.}
T=$(mktemp -d)
cp "$lib" $T/lib.so
(cd $T && /opt/rocm/llvm/bin/llvm-objdump --offloading lib.so > /dev/null)
for o in $T/*gfx950; do
  /opt/rocm/llvm/bin/llvm-readelf --notes "$o" | awk '
    /^ +- \.agpr_count/ {a=$NF}
    /\.name: +_Z/ {n=$NF}
    /\.private_segment_fixed_size:/ {p=$NF}
    /\.vgpr_count:/ {v=$NF}
    /\.vgpr_spill_count:/ {s=$NF; print n, "vgpr=" v, "scratch=" p, "vspill=" s}'
done | c++filt | grep -E "$filt"
rm -rf $T
