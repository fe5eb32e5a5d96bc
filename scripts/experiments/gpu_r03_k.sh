#!/bin/bash
# Round 3: band-first overlap over the host-staged transport with ONE rank
# (periodic domain: the faces go D2H -> MPI to itself -> H2D while the GPU
# would otherwise idle), serial / band-first / auto, three repetitions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$PWD
OUT=$R/gpurun_out/r03_k
mkdir -p $OUT
: > $OUT/mpihost1.txt
for rep in 1 2 3; do
  for n in 16384 8192; do
    for mode in "--no-overlap" "--overlap" "--overlap=auto"; do
      timeout -k 10 200 build/bin/mpi_jacobi2d $n 100 --tblock --tsteps=20 --warmup=20 --periodic \
        --transport=mpi-host $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
      echo "rep=$rep n=$n [$mode] $(grep -E 'TIME step|overlap|halo' $OUT/j.log | tr '\n' ' ')" | tee -a $OUT/mpihost1.txt
    done
  done
done
