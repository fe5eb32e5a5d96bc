#!/bin/bash
# K = 14 sweeps per pass: numerics, engine checks, bench K=12 vs 14, shares.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/k14
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -m gpu -x -q -k "jacobi5xk or engine or app_jacobi" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
M=/opt/conda/bin/mpirun
for K in 12 14; do
  timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d 515 37 --check --periodic --transport=rccl --tblock --tsteps=$K --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
  grep -E "check" $OUT/jc.log
  timeout -k 10 120 $M -np 4 build/bin/mpi_jacobi2d 515 37 --check --tblock --tsteps=$K --dims=2x2 --transport=ipc --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
  grep -E "check" $OUT/jc.log
done
for K in 12 14; do
  for run in 1 2; do
    timeout -k 10 300 python bench.py --tsteps $K --skip-extras > $OUT/bench$K.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    echo "K=$K $(python3 -c "import json; r=json.load(open('$OUT/bench$K.json')); print(r['value'], r['ms_per_step'])")"
  done
done
for cfg in "16384 32768" "8192 32768" "8192 16384"; do
  set -- $cfg
  for K in 12 14; do
    timeout -k 10 200 $M -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 84 --tblock --tsteps=$K --warmup=$K --periodic --transport=rccl > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "ny=$1 nx=$2 K=$K $(grep -E 'TIME step' $OUT/j.log)"
  done
done
