#!/bin/bash
# Round 6 (u): where the dispatcher puts the waves of the K-sweep kernel's
# workgroup shapes (build/bench/wave_place: one, two and four two-stage
# strips per workgroup at 28 KB of LDS per strip, 256 VGPRs per lane).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=$PWD/gpurun_out/r06_u
mkdir -p $OUT
for nw in 1 2 4; do
  timeout -k 10 60 build/bench/wave_place $nw 28 > $OUT/place_nw$nw.txt 2>&1 || { cat $OUT/place_nw$nw.txt; exit 1; }
  cat $OUT/place_nw$nw.txt
done
echo R06U_OK
