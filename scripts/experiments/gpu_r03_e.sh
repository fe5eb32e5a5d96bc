#!/bin/bash
# Round 3: (1) band-first overlap over the host-staged transport (2 ranks on
# one GPU, mpi-host: an exchange of ~1 ms that overlap can hide); (2) kernel
# traces of the two N = 8 shares (4x2: 8192 x 16384, 2x4: 16384 x 8192),
# Dirichlet sides, 100 sweeps, to split pass time / launch gaps / clock drift.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/r03_e
mkdir -p $OUT
M=/opt/conda/bin/mpirun
: > $OUT/mpihost.txt
for n in 8192 16384; do
  for mode in "--no-overlap" "--overlap" "--overlap=auto"; do
    timeout -k 10 200 $M -np 2 $R/build/bin/mpi_jacobi2d $n 100 --tblock --tsteps=20 --warmup=20 \
      --transport=mpi-host $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "n=$n [$mode] $(grep -E 'TIME step|overlap' $OUT/j.log | tr '\n' ' ')" | tee -a $OUT/mpihost.txt
  done
done
cd /tmp
for sh in "8192 16384" "16384 8192"; do
  set -- $sh
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_$1x$2 -o t -- \
    $R/build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 --graph > $OUT/tr_$1x$2.log 2>&1 || { tail -30 $OUT/tr_$1x$2.log; exit 1; }
  grep -E "TIME step" $OUT/tr_$1x$2.log
done
echo DONE
