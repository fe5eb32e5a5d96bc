#!/bin/bash
# A/B of kernel variants on one box (build/var/*/libgmt.so via LD_LIBRARY_PATH),
# sustained K = 20 at 32768^2 and the N = 8 share, alternating twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
B=build/bin/gmt_kernel_bench
for rep in 1 2; do
  for v in base "$@"; do
    lp=""; [ "$v" != base ] && lp=build/var/$v
    LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --iters=20 --tb-k=20 --tb-mask=0 --jacobi-n=32768 > $OUT/$v.log 2>&1 || { cat $OUT/$v.log; exit 1; }
    LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --iters=100 --tb-k=20 --tb-mask=0 --jacobi-ny=8192 --jacobi-nx=16384 >> $OUT/$v.log 2>&1 || { cat $OUT/$v.log; exit 1; }
    echo "$v: $(grep MLUPS $OUT/$v.log | awk '{print $(NF-13)}' | tr '\n' ' ') $(grep -o 'vgpr [0-9]*' $OUT/$v.log | head -1)"
  done
done
