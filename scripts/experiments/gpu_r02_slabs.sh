#!/bin/bash
# row-slab shares (choose_dims picks 4x1 at N = 4; 8x1 is the alternative at N = 8)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/slabs}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
for cfg in "8192 32768" "4096 32768" "8192 16384"; do
  set -- $cfg
  for mode in "" "--periodic --transport=rccl --overlap=auto"; do
    timeout -k 10 200 $M -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 --graph $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log)"
  done
done
