#!/bin/bash
# per-GPU strong-scaling shares at the bench defaults (K = 14, scaled levels)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/share14
mkdir -p $OUT
M=/opt/conda/bin/mpirun
for cfg in "32768 32768" "16384 32768" "8192 32768" "8192 16384"; do
  set -- $cfg
  for mode in "" "--periodic --transport=rccl" "--periodic --transport=rccl --no-overlap"; do
    timeout -k 10 200 $M -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=14 --warmup=14 $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log)"
  done
done
