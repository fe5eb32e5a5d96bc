#!/bin/bash
# Round 5 (y): edge segments dispatched last on every XCD (GMT_TB_EDGES_LAST=1,
# tail_swizzle; the planner models the order and may pick short edges) vs the
# default order, Dirichlet domains; numerics of the new order first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_y
mkdir -p $OUT
GMT_TB_EDGES_LAST=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jacobi_tb_gpu.py \
  tests/test_push_gpu.py -k "not ranks_sharing" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60"; do
    for el in 0 1; do
      echo "== el$el $shp" >> $OUT/rates.log
      GMT_TB_EDGES_LAST=$el timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
