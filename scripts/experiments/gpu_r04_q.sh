#!/bin/bash
# Round 4 (q): segment count sweep on single-round shares (fewer workgroups
# than resident slots: do the under-filled CUs run their waves faster than
# the makespan model assumes?) and on 32768^2 (8 rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_q}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/seg.txt
run() {  # mask shape segs
  timeout -k 10 300 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$1 $2 --tb-seg=$3 > $OUT/s.log 2>&1 || { cat $OUT/s.log; exit 1; }
  grep MLUPS $OUT/s.log | tee -a $OUT/seg.txt
}
for rep in 1 2; do
  run 15 "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" 0,631,683,745,820,911
  run 15 "--jacobi-ny=16384 --jacobi-nx=8192 --iters=100" 0,656,683,713,745,820
  run 15 "--jacobi-n=8192 --iters=100" 0,342,357,373,410,456
  run 0 "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" 0,683,745,820,911
  run 0 "--jacobi-n=8192 --iters=100" 0,357,373,410,456
  run 0 "--jacobi-n=32768 --iters=20" 0,600,680,720,800
done
