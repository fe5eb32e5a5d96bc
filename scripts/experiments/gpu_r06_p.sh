#!/bin/bash
# Round 6 (p): same box, alternating: per-strip launch, one strip per
# workgroup (nw1); two strips per workgroup with stage-major waves (nw2m1);
# shared hand-off groups (sh, the default where it applies).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_p
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
    for mask in 0 15; do
      for v in nw1 nw2m1 sh; do
        case $v in
          nw1) envs="GMT_TB_SHARED=0"; nw=0;;
          nw2m1) envs="GMT_TB_SHARED=0 GMT_TB_STRIP_MAP=1"; nw=2;;
          sh) envs="GMT_TB_SHARED=1"; nw=0;;
        esac
        echo "== $v m$mask $shp" >> $OUT/rates.log
        env $envs timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-nw=$nw --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
echo R06P_OK
