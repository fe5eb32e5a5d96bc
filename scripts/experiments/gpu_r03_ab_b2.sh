#!/bin/bash
# Round 3 A/B: two-stage strips with one s_barrier every 2 steps (build/var/b2)
# vs the production kernel: bitwise checks first, then sustained K = 20
# rates on the full domain and the strong-scaling shares, twice, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/r03_ab_b2}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
for k in 12 14 20; do
  LD_LIBRARY_PATH=build/var/b2 timeout -k 10 120 build/bin/mpi_jacobi2d --ny=700 --nx=1900 0 47 --check --tblock --tsteps=$k \
    --periodic 2>&1 | grep -E "check" || { echo "check K=$k failed"; exit 1; }
  LD_LIBRARY_PATH=build/var/b2 timeout -k 10 120 build/bin/mpi_jacobi2d --ny=700 --nx=1900 0 47 --check --tblock --tsteps=$k \
    2>&1 | grep -E "check" || { echo "check K=$k failed"; exit 1; }
done
LD_LIBRARY_PATH=build/var/b2 timeout -k 10 120 $M -np 2 build/bin/mpi_jacobi2d --ny=701 --nx=1900 0 47 --check --tblock --tsteps=20 \
  --transport=ipc --dims=2x1 2>&1 | grep -E "check" || { echo "check 2 ranks failed"; exit 1; }
B=build/bin/gmt_kernel_bench
for rep in 1 2; do
  for v in base b2; do
    lp=""; [ "$v" != base ] && lp=build/var/$v
    : > $OUT/$v.$rep.log
    for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=16384 --jacobi-nx=32768 --iters=40" "--jacobi-n=16384 --iters=60" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=100" "--jacobi-n=8192 --iters=100"; do
      LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/$v.$rep.log 2>&1 || { cat $OUT/$v.$rep.log; exit 1; }
    done
    echo "$v: $(grep MLUPS $OUT/$v.$rep.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
  done
done
