#!/bin/bash
# Round 4 (x): a deliberately exposed exchange: 1 rank, periodic, host-staged
# (mpi-host) on 16384^2 and 8192 x 16384.  Serial vs band-first vs
# --overlap=auto (which order the autotune keeps), 3 alternating reps; the
# app's "halo" line is the blocking exchange alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_x}
mkdir -p $OUT
MPI=/opt/conda/bin/mpirun
: > $OUT/summary.txt
for rep in 1 2 3; do
  for cfg in "16384 16384" "8192 16384"; do
    set -- $cfg
    for mode in "--no-overlap" "--overlap" "--overlap=auto"; do
      timeout -k 10 200 $MPI -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 \
        --periodic --transport=mpi-host $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
      echo "rep=$rep ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log) | $(grep -E '^transport' $OUT/j.log) | $(grep -E '^halo' $OUT/j.log)" | tee -a $OUT/summary.txt
    done
  done
done
