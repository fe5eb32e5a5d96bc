#!/bin/bash
# Round 4 (p): does the single-round tail cost what the makespan model says?
# Forced segment lengths on the N = 8 shares and 8192^2 (1 round = the
# planner's choice, vs 2, 3, 4 rounds of shorter segments), mask 15 and 0.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_p}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/seg.txt
for rep in 1 2; do
  for m in 15 0; do
    for shp in "--jacobi-ny=8192 --jacobi-nx=16384" "--jacobi-ny=16384 --jacobi-nx=8192" "--jacobi-n=8192"; do
      timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$m --iters=100 $shp --tb-seg=0,480,360,240,180,120 \
        > $OUT/s.log 2>&1 || { cat $OUT/s.log; exit 1; }
      grep MLUPS $OUT/s.log | sed "s/^/rep=$rep /" | tee -a $OUT/seg.txt
    done
  done
done
