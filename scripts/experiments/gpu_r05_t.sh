#!/bin/bash
# Round 5 (t): which sweep count's band-first pass never signals at 2 ranks
# sharing the GPU (bench.py's start-up calibration runs every K band-first)?
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_t
mkdir -p $OUT
M=/opt/conda/bin/mpirun
B=$R/build/bin/mpi_jacobi2d
for K in 2 3 4 5 6 7 8 9 10 12 14 16 18 20; do
  timeout -k 10 60 $M -np 2 $B 0 $((3 * K)) --ny=8192 --nx=8192 --dims=2x1 --tblock --tsteps=$K --transport=ipc --warmup=0 \
    > $OUT/k$K.log 2>&1
  rc=$?
  echo "K $K rc $rc $(grep -E 'timed out|TIME step' $OUT/k$K.log | head -1)"
  [ $rc -ge 124 ] && exit 1
done
echo R05T_OK
