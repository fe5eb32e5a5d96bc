#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/xk
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "jacobi5x" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
M=/opt/conda/bin/mpirun
for K in 3 4; do
  for a in "515 31 --check" "515 30 --check --periodic --graph --transport=rccl"; do
    timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d $a --tblock --tsteps=$K --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
    grep -E "check" $OUT/jc.log
  done
  timeout -k 10 120 $M -np 4 build/bin/mpi_jacobi2d 515 30 --check --tblock --tsteps=$K --dims=2x2 --periodic --transport=ipc --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
  grep -E "check" $OUT/jc.log
done
timeout -k 10 400 build/bin/gmt_kernel_bench --iters=10 --only=jacobi --jacobi-n=32768 > $OUT/kb32k.log 2>&1 || { cat $OUT/kb32k.log; exit 1; }
grep -E "xk|v9" $OUT/kb32k.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
