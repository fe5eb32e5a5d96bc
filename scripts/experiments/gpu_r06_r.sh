#!/bin/bash
# Round 6 (r): where the two-strip default should start — 16384^2 (two
# rounds, the N = 4 share) and the N = 2 shares, one vs two strips per
# workgroup, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_r
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=16384 --iters=40" "--jacobi-ny=16384 --jacobi-nx=32768 --iters=20" "--jacobi-ny=32768 --jacobi-nx=16384 --iters=20"; do
    for mask in 0 5 15; do
      for nw in 1 2; do
        echo "== nw$nw m$mask $shp" >> $OUT/rates.log
        GMT_TB_SHARED=0 timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-nw=$nw --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
echo R06R_OK
