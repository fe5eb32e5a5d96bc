#!/bin/bash
# Multiply-free scaled levels in the pipelined fast path: numerics + A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/scaled
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -m gpu -x -q -k "jacobi5xk or engine or app_jacobi" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
M=/opt/conda/bin/mpirun
for K in 8 10 12 14; do
  for S in 0 1; do
    timeout -k 10 200 env GMT_PIPE_SCALED=$S $M -np 1 build/bin/mpi_jacobi2d 32768 $((K*4)) --tblock --tsteps=$K --warmup=$K > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "K=$K scaled=$S $(grep -E 'TIME step' $OUT/j.log)"
  done
done
for S in 0 1 0 1; do
  timeout -k 10 300 env GMT_PIPE_SCALED=$S python bench.py --skip-extras > $OUT/bench$S.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  echo "bench scaled=$S $(python3 -c "import json; r=json.load(open('$OUT/bench$S.json')); print(r['value'], r['ms_per_step'])")"
done
