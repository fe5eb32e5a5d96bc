#!/bin/bash
# Skewed register pipeline: numerics + engine checks + occupancy/segment sweep + bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pipe4
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "jacobi5x" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
M=/opt/conda/bin/mpirun
for K in 6 8; do
  timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d 515 30 --check --periodic --graph --transport=rccl --tblock --tsteps=$K --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
  grep -E "check" $OUT/jc.log
  timeout -k 10 120 $M -np 4 build/bin/mpi_jacobi2d 515 30 --check --tblock --tsteps=$K --dims=2x2 --periodic --transport=ipc --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
  grep -E "check" $OUT/jc.log
done
timeout -k 10 400 build/bin/gmt_kernel_bench --iters=10 --only=jacobi --sections=pipe --jacobi-n=32768 > $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
grep -E "pipe" $OUT/kb.log
timeout -k 10 300 python bench.py --tsteps 8 > $OUT/bench8.json 2> $OUT/bench8.err || { tail -20 $OUT/bench8.err; exit 1; }
cat $OUT/bench8.json
timeout -k 10 300 python bench.py --tsteps 6 > $OUT/bench6.json 2> $OUT/bench6.err || { tail -20 $OUT/bench6.err; exit 1; }
cat $OUT/bench6.json
