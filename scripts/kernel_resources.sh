#!/bin/bash
# Compile-time register/occupancy report of a HIP source for gfx950:
#   scripts/kernel_resources.sh csrc/kernels/jacobi5pipe.hip [name-filter]
f=$1; filt=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Icsrc/include -munsafe-fp-atomics \
  -c "$f" -o /tmp/kr.$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy" |
  sed -E 's/.*remark: *//; s/ \[-Rpass.*//' | paste - - - - - | grep -E "$filt" |
  sed -E 's/Function Name: //' | c++filt | awk -F'\t' '{printf "%-70.70s %s %s %s %s\n",$1,$2,$3,$4,$5}'
rm -f /tmp/kr.$$.o
