#!/bin/bash
# Round 5 (j): push-aware segment plans + chunk-ordered host staging.
#   1. push / TB / staging-kernel tests;
#   2. kernel level: push pass vs plain pass, alternated (GMT_TB_PUSH_COST 1.15 default, 1.3);
#   3. app level: serial RCCL vs inline halo, one rank periodic, 2000 steps;
#   4. mpi-host 8 MiB and the reference's stage_host exchange, traced, with MPI alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_j
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_push_gpu.py \
  tests/test_jacobi_tb_gpu.py "tests/test_kernels_gpu.py::test_stage_gather_scatter_field_blocks" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=$R/build/bin
: > $OUT/kpush.log
for c in 1.15 1.3; do
  for shp in "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60" "--jacobi-n=32768 --iters=20"; do
    echo "== c$c $shp" >> $OUT/kpush.log
    GMT_TB_PUSH_COST=$c timeout -k 10 200 $B/gmt_kernel_bench --only=tb --sustained=1 --tb-k=20 --tb-mask=15 --tb-push=1 $shp >> $OUT/kpush.log 2>&1 || { tail -20 $OUT/kpush.log; exit 1; }
  done
done
grep -E "^==|ratio" $OUT/kpush.log
MPIRUN=/opt/conda/bin/mpirun
: > $OUT/app.log
for rep in 1 2; do
  for shp in "--ny=8192 --nx=16384" "--ny=16384 --nx=8192"; do
    for mode in "serial:--no-overlap" "push:--push"; do
      name=${mode%%:*}; opts=${mode#*:}
      echo "== $name $shp" >> $OUT/app.log
      timeout -k 10 120 $MPIRUN -np 1 $B/mpi_jacobi2d 0 2000 $shp --periodic --tblock --tsteps=20 \
        --warmup=100 --transport=rccl $opts >> $OUT/app.log 2>&1 || { tail -20 $OUT/app.log; exit 1; }
    done
  done
done
grep -E "^==|TIME step" $OUT/app.log
OUT=gpurun_out/r05_j/xport bash scripts/experiments/gpu_r05_e.sh
