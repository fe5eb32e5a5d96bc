#!/bin/bash
# pass costs of the 4-column kernel (sustained, every K) at 32768^2 and 8192^2
# -> JacobiSolver's kCostLarge / kCostSmall tables
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/costs3}
mkdir -p $OUT
KS=1,2,3,4,5,6,7,8,9,10,12,14,16,18,20,22,24
timeout -k 10 300 build/bin/gmt_kernel_bench --only=tb --tb-k=$KS --jacobi-n=32768 --iters=8 --sustained=1 \
  > $OUT/costs_32768.log 2>&1 || { tail -5 $OUT/costs_32768.log; exit 1; }
grep " ms" $OUT/costs_32768.log
timeout -k 10 300 build/bin/gmt_kernel_bench --only=tb --tb-k=$KS --jacobi-n=8192 --iters=40 --sustained=1 \
  > $OUT/costs_8192.log 2>&1 || { tail -5 $OUT/costs_8192.log; exit 1; }
grep " ms" $OUT/costs_8192.log
