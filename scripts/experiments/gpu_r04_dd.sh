#!/bin/bash
# Round 4 (dd): band-first vs serial with the one-kernel in-place IPC
# exchange, 2 ranks sharing the GPU (16384^2 and 16384 x 32768), 3 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_dd}
mkdir -p $OUT
MPI=/opt/conda/bin/mpirun
: > $OUT/summary.txt
for rep in 1 2 3; do
  for cfg in "16384 16384" "16384 32768"; do
    set -- $cfg
    for mode in "--no-overlap" "--overlap"; do
      timeout -k 10 200 $MPI -np 2 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 \
        --periodic --transport=ipc $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
      echo "rep=$rep ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log) | $(grep -E '^transport' $OUT/j.log)" | tee -a $OUT/summary.txt
    done
  done
done
