#!/bin/bash
# Round 6 (t): the stage-0 priority (GMT_TB_PRIO=1: s_setprio(2) on every
# stage-0 wave, multi-round launches too) against the default, with one and
# two strips per workgroup (stage-major) and three, same box, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_t
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=16384 --jacobi-nx=32768 --iters=20"; do
    for mask in 0 15; do
      for v in nw1 nw1p nw2 nw2p nw3; do
        case $v in
          nw1) envs="GMT_TB_SHARED=0"; nw=1;;
          nw1p) envs="GMT_TB_SHARED=0 GMT_TB_PRIO=1"; nw=1;;
          nw2) envs="GMT_TB_SHARED=0"; nw=2;;
          nw2p) envs="GMT_TB_SHARED=0 GMT_TB_PRIO=1"; nw=2;;
          nw3) envs="GMT_TB_SHARED=0"; nw=3;;
        esac
        echo "== $v m$mask $shp" >> $OUT/rates.log
        env $envs timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-nw=$nw --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
echo R06T_OK
