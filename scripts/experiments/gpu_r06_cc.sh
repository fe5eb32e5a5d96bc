#!/bin/bash
# Round 6 (cc): the 2^28-point shapes (the N = 4 shares: 8192 x 32768 for a
# 4 x 1 grid, 16384^2 for 2 x 2) — one strip (the default at 2^28), two plain
# stage-major strips, two-strip shared groups; same box, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_cc
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-ny=8192 --jacobi-nx=32768 --iters=40" "--jacobi-n=16384 --iters=40"; do
    for mask in 12 0 5; do
      for v in nw1 nw2 sh2; do
        case $v in
          nw1) envs="GMT_TB_SHARED=0"; nw=1;;
          nw2) envs="GMT_TB_SHARED=0"; nw=2;;
          sh2) envs="GMT_TB_SHARED=2"; nw=0;;
        esac
        echo "== $v m$mask $shp" >> $OUT/rates.log
        env $envs timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-nw=$nw --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
echo R06CC_OK
