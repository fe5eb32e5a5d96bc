#!/bin/bash
# Round 5 (g): the exec-masked Dirichlet keep with its skip branch
#   1. TB bitwise tests (Dirichlet rule paths) + push kernel tests;
#   2. rates new / nobr (keep without the skip branch) / head (per-cell select);
#   3. where the app's pass time goes: mpi_jacobi2d one rank, periodic,
#      serial vs inline halo at 2000 steps, and a kernel trace of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_g
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jacobi_tb_gpu.py \
  tests/test_push_gpu.py -k "not ranks_sharing" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=$R/build/bin
MPIRUN=/opt/conda/bin/mpirun
: > $OUT/app.log
for mode in "serial:--no-overlap" "push:--push"; do
  name=${mode%%:*}; opts=${mode#*:}
  for st in 2000 200; do
    echo "== $name steps $st" >> $OUT/app.log
    timeout -k 10 120 $MPIRUN -np 1 $B/mpi_jacobi2d 0 $st --ny=8192 --nx=16384 --periodic --tblock --tsteps=20 \
      --warmup=40 --transport=rccl $opts >> $OUT/app.log 2>&1 || { tail -20 $OUT/app.log; exit 1; }
  done
  timeout -k 10 180 $MPIRUN -np 1 rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o $name -- \
    $B/mpi_jacobi2d 0 400 --ny=8192 --nx=16384 --periodic --tblock --tsteps=20 --warmup=40 --transport=rccl $opts \
    > $OUT/prof_$name.log 2>&1 || { tail -20 $OUT/prof_$name.log; exit 1; }
done
grep -E "^==|TIME step" $OUT/app.log
OUT=gpurun_out/r05_g VARIANTS="new nobr head" bash scripts/experiments/gpu_r05_d.sh
