#!/bin/bash
# Round 6 (v): one-round launches — the stage-0 priority they get by default
# (a.prio) against none (GMT_TB_PRIO=0), one strip and two stage-major strips
# per workgroup, same box, alternating; then the wave placement probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_v
mkdir -p $OUT
for nw in 1 2 4; do
  timeout -k 10 60 build/bench/wave_place $nw 28 > $OUT/place_nw$nw.txt 2>&1 || { cat $OUT/place_nw$nw.txt; exit 1; }
  cat $OUT/place_nw$nw.txt
done
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
    for mask in 0 15; do
      for v in nw1 nw1p0 nw2 nw2p0; do
        case $v in
          nw1) envs="GMT_TB_SHARED=0"; nw=1;;
          nw1p0) envs="GMT_TB_SHARED=0 GMT_TB_PRIO=0"; nw=1;;
          nw2) envs="GMT_TB_SHARED=0"; nw=2;;
          nw2p0) envs="GMT_TB_SHARED=0 GMT_TB_PRIO=0"; nw=2;;
        esac
        echo "== $v m$mask $shp" >> $OUT/rates.log
        env $envs timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-nw=$nw --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
echo R06V_OK
