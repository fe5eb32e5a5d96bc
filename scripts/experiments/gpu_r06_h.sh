#!/bin/bash
# Round 6 (h): the first block of the K >= 12 second stage skipped (all its
# levels dead: GMT_TB_SKIP_DEAD) — bitwise tests, then same-box A/B against
# the variant build without it (build/var/noskip), alternating, Dirichlet
# and halo sides, the BASELINE domains and the N = 8 shares.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_jacobi_tb_gpu.py tests/test_push_gpu.py tests/test_production_geometry_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2 3; do
  for shp in "--jacobi-n=8192 --iters=200" "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
    for mask in 0 15; do
      for v in skip noskip; do
        echo "== $v m$mask $shp" >> $OUT/rates.log
        if [ $v = noskip ]; then
          LD_LIBRARY_PATH=$R/build/var/noskip timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
        else
          timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
        fi
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
echo R06H_OK
