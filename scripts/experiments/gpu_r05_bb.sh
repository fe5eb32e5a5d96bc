#!/bin/bash
# Round 5 (bb): push cost 1.3 as the default — push numerics, kernel-level
# push/plain ratios and the application against the serial order.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_bb
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_push_gpu.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=$R/build/bin
: > $OUT/kpush.log
for shp in "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
  echo "== $shp" >> $OUT/kpush.log
  timeout -k 10 200 $B/gmt_kernel_bench --only=tb --sustained=1 --tb-k=20 --tb-mask=15 --tb-push=1 $shp >> $OUT/kpush.log 2>&1 || { tail -20 $OUT/kpush.log; exit 1; }
done
grep -E "^==|ratio" $OUT/kpush.log
M=/opt/conda/bin/mpirun
: > $OUT/app.log
for rep in 1 2 3; do
  for shp in "--ny=8192 --nx=16384" "--ny=16384 --nx=8192"; do
    for mode in "serial:--no-overlap" "push:--push"; do
      name=${mode%%:*}; opts=${mode#*:}
      echo "== $name $shp" >> $OUT/app.log
      timeout -k 10 120 $M -np 1 $B/mpi_jacobi2d 0 2000 $shp --periodic --tblock --tsteps=20 --warmup=100 \
        --transport=rccl $opts >> $OUT/app.log 2>&1 || { tail -20 $OUT/app.log; exit 1; }
    done
  done
done
grep -E "^==|TIME step" $OUT/app.log | paste - - | awk '{print $2, $3, $4, $(NF-1)}'
