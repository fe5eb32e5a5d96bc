#!/bin/bash
# Strong-scaling shares of the 32768^2 bench on ONE GPU (tsteps 20): each
# share's time without any exchange (Dirichlet), with a 1-rank periodic RCCL
# self-exchange of all four K-wide faces overlapped / serial / autotuned.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/shares}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
K=${K:-20}
for cfg in "32768 32768" "16384 32768" "16384 16384" "8192 16384" "16384 8192"; do
  set -- $cfg
  for mode in "" "--periodic --transport=rccl" "--periodic --transport=rccl --no-overlap" "--periodic --transport=rccl --overlap=auto"; do
    timeout -k 10 200 $M -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=$K --warmup=$K --graph $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "ny=$1 nx=$2 [$mode] $(grep -E 'TIME step|overlap' $OUT/j.log | tr '\n' ' ')"
  done
done
