#!/bin/bash
# Round 5 (b): the cheap Dirichlet row rule (uniform per-level branch, ring
# rows / columns only, no edge segments) against HEAD's kernel, same box,
# alternating; then the bitwise kernel tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r05_b}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for v in new head; do
    lp=""; [ "$v" != new ] && lp=$R/build/var/$v
    for m in 0 15; do
      for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60"; do
        echo "== $v m$m $shp" >> $OUT/rates.log
        LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$m $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $(NF-13), $(NF-12)}' | sed 's/MLUPS//'
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jacobi_tb_gpu.py > $OUT/pytest_tb.log 2>&1 || { tail -40 $OUT/pytest_tb.log; exit 1; }
tail -2 $OUT/pytest_tb.log
