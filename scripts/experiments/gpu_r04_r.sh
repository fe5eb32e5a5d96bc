#!/bin/bash
# Round 4 (r): is the first configuration of a gmt_kernel_bench invocation
# slow (order effect), or is the planner's own plan slower than the same
# segment length forced?  Alternate seg=0 and the forced length.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_r}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/seg.txt
run() {
  timeout -k 10 300 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$1 $2 --tb-seg=$3 > $OUT/s.log 2>&1 || { cat $OUT/s.log; exit 1; }
  grep MLUPS $OUT/s.log | tee -a $OUT/seg.txt
}
run 15 "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" 631,0,631,0
run 15 "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" 0,631,0,631
run 15 "--jacobi-n=8192 --iters=100" 357,0,357,0
run 15 "--jacobi-n=8192 --iters=100" 0,357,0,357
run 0 "--jacobi-n=32768 --iters=20" 0,0,0
run 0 "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" 0,0,0
