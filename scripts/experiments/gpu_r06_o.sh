#!/bin/bash
# Round 6 (o): per-strip launches (GMT_TB_SHARED=0) with several two-stage
# strips per workgroup and stage-major waves (GMT_TB_STRIP_MAP=1): does the
# SIMD balance that made the shared groups fast help the one-round 8192^2
# and N = 8 share passes?  Bitwise tests of the multi-strip shapes first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_o
mkdir -p $OUT
GMT_TB_STRIP_MAP=1 timeout -k 10 600 python -u -m pytest tests/test_jacobi_tb_gpu.py -x -q -k "workgroup_shapes or bitwise" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60" "--jacobi-n=32768 --iters=20"; do
    for mask in 0 15; do
      for v in nw1 nw4m0 nw4m1 nw2m1; do
        case $v in
          nw1) envs="GMT_TB_SHARED=0"; nw=1;;
          nw4m0) envs="GMT_TB_SHARED=0"; nw=4;;
          nw4m1) envs="GMT_TB_SHARED=0 GMT_TB_STRIP_MAP=1"; nw=4;;
          nw2m1) envs="GMT_TB_SHARED=0 GMT_TB_STRIP_MAP=1"; nw=2;;
        esac
        echo "== $v m$mask $shp" >> $OUT/rates.log
        env $envs timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-nw=$nw --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
echo R06O_OK
