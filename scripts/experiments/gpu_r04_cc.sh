#!/bin/bash
# Round 4 (cc): the makespan model's segment length vs forced ones with the
# model's rule/edge handling kept (GMT_TB_PLAN_L), headline pass (32768^2,
# Dirichlet) and 8192^2 / 8192 x 16384 Dirichlet, warmed harness, 2 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_cc}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/l.txt
run() {  # L shape
  GMT_TB_PLAN_L=$1 timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $2 > $OUT/s.log 2>&1 || { cat $OUT/s.log; exit 1; }
  grep MLUPS $OUT/s.log | sed "s/^/L=$1 /" | tee -a $OUT/l.txt
}
for rep in 1 2; do
  for L in 0 800 900 1100 1250 1640; do run $L "--jacobi-n=32768 --iters=20"; done
  for L in 0 300 400 450; do run $L "--jacobi-n=8192 --iters=100"; done
  for L in 0 600 680 820; do run $L "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100"; done
done
