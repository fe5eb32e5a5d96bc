#!/bin/bash
# K = 10/12 sweeps per pass: numerics, engine checks, kernel A/B, bench per K.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/k12${TAG:-}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "jacobi5xk" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
M=/opt/conda/bin/mpirun
for K in 8 10 12; do
  timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d 515 37 --check --periodic --graph --transport=rccl --tblock --tsteps=$K --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
  grep -E "check" $OUT/jc.log
  timeout -k 10 120 $M -np 4 build/bin/mpi_jacobi2d 515 37 --check --tblock --tsteps=$K --dims=2x2 --periodic --transport=ipc --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
  grep -E "check" $OUT/jc.log
done
timeout -k 10 400 build/bin/gmt_kernel_bench --iters=10 --only=jacobi --sections=pipe --jacobi-n=32768 > $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
grep -E "pipe v(8|10|12) " $OUT/kb.log
for K in 8 10 12; do
  timeout -k 10 300 python bench.py --tsteps $K --skip-extras > $OUT/bench$K.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench$K.json
done
