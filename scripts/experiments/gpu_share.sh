#!/bin/bash
# (1) the native-layer GPU tests (engine in-process + HIP apps under MPICH);
# (2) per-GPU share of the strong-scaling bench on one MI355X: the local
#     domain rank r would own at N = 2/4/8 (bench.py grid: 2x1, 4x1, 4x2 of
#     32768^2), run as one periodic rank that exchanges all four 12-wide halos
#     with itself through RCCL every pass (an upper bound on a real rank's
#     exchange work), eager (N>1 bench mode) and graph.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/share
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_native_gpu.log 2>&1 || { tail -40 $OUT/pytest_native_gpu.log; exit 1; }
tail -2 $OUT/pytest_native_gpu.log
M=/opt/conda/bin/mpirun
J=--json=$OUT/share.jsonl
for cfg in "32768 32768" "16384 32768" "8192 32768" "8192 16384"; do
  set -- $cfg
  for mode in "" "--periodic --transport=rccl" "--periodic --transport=rccl --graph"; do
    timeout -k 10 200 $M -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 60 --tblock --tsteps=12 --warmup=12 $mode $J > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "ny=$1 nx=$2 [$mode] $(grep -E 'TIME step|MLUPS' $OUT/j.log | tr '\n' ' ')"
  done
done
