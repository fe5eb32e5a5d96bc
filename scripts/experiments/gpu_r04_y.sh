#!/bin/bash
# Round 4 (y): the headline pass (32768^2, Dirichlet sides) with the planner's
# segment length vs longer forced ones, warmed harness, 2 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_y}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/seg.txt
for rep in 1 2; do
  timeout -k 10 300 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 --jacobi-n=32768 --iters=20 \
    --tb-seg=0,1100,1260,1400,1640,2048,0 > $OUT/s.log 2>&1 || { cat $OUT/s.log; exit 1; }
  grep MLUPS $OUT/s.log | sed "s/^/rep=$rep /" | tee -a $OUT/seg.txt
done
