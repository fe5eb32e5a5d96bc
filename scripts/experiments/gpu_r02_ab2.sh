#!/bin/bash
# A/B over the strong-scaling share shapes too (K = 20, Dirichlet), twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/ab2}
mkdir -p $OUT
B=build/bin/gmt_kernel_bench
for rep in 1 2; do
  for v in base "$@"; do
    lp=""; [ "$v" != base ] && lp=build/var/$v
    : > $OUT/$v.log
    for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=16384 --jacobi-nx=32768 --iters=40" "--jacobi-n=16384 --iters=60" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" "--jacobi-n=8192 --iters=100"; do
      LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/$v.log 2>&1 || { cat $OUT/$v.log; exit 1; }
    done
    echo "$v: $(grep MLUPS $OUT/$v.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
  done
done
