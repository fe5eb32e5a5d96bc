#!/bin/bash
# Register-pipelined K-sweep kernel: numerics (pytest), engine --check for
# K = 2..8 on the local, RCCL-periodic and IPC 2x2 paths, kernel bench, bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pipe
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "jacobi5x" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
M=/opt/conda/bin/mpirun
for K in 2 4 6 8; do
  for a in "515 31 --check" "515 30 --check --periodic --graph --transport=rccl"; do
    timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d $a --tblock --tsteps=$K --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
    grep -E "check" $OUT/jc.log
  done
  timeout -k 10 120 $M -np 4 build/bin/mpi_jacobi2d 515 30 --check --tblock --tsteps=$K --dims=2x2 --periodic --transport=ipc --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
  grep -E "check" $OUT/jc.log
done
timeout -k 10 400 build/bin/gmt_kernel_bench --iters=10 --only=jacobi --jacobi-n=32768 > $OUT/kb32k.log 2>&1 || { cat $OUT/kb32k.log; exit 1; }
grep -E "xk|v9|pipe" $OUT/kb32k.log
for K in 4 8; do
  timeout -k 10 300 python bench.py --tsteps $K > $OUT/bench$K.json 2> $OUT/bench$K.err || { tail -20 $OUT/bench$K.err; exit 1; }
  cat $OUT/bench$K.json
done
