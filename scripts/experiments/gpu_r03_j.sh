#!/bin/bash
# Round 3: (1) the dim-1 derivative, d1_walk harness vs gmt_kernel_bench (the
# production entry point) on one box; (2) band-first over the host-staged
# transport, 2 ranks on one GPU, 16384^2 and 12288^2, three alternating
# repetitions of serial / band-first / auto.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$PWD
OUT=$R/gpurun_out/r03_j
mkdir -p $OUT
timeout -k 10 300 build/bench/d1_walk > $OUT/d1_walk.txt 2>&1 || { cat $OUT/d1_walk.txt; exit 1; }
head -3 $OUT/d1_walk.txt
timeout -k 10 120 build/bin/gmt_kernel_bench --only=stencil > $OUT/deriv.txt 2>&1 && tail -3 $OUT/deriv.txt
timeout -k 10 120 build/bin/gmt_kernel_bench --only=stencil --sustained=1 --iters=20 > $OUT/deriv_sus.txt 2>&1 && tail -2 $OUT/deriv_sus.txt
M=/opt/conda/bin/mpirun
: > $OUT/mpihost.txt
for rep in 1 2 3; do
  for n in 16384 12288; do
    for mode in "--no-overlap" "--overlap" "--overlap=auto"; do
      timeout -k 10 200 $M -np 2 $R/build/bin/mpi_jacobi2d $n 100 --tblock --tsteps=20 --warmup=20 \
        --transport=mpi-host $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
      echo "rep=$rep n=$n [$mode] $(grep -E 'TIME step|overlap|halo' $OUT/j.log | tr '\n' ' ')" | tee -a $OUT/mpihost.txt
    done
  done
done
