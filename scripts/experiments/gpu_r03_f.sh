#!/bin/bash
# Round 3: lane shifts through ds_bpermute (LDS crossbar, off the VALU) vs
# DPP moves in the temporal-blocking kernel (build/var/bp), and the no-shift
# upper bound (build/var/ns: wrong results, timing only); dim-1 derivative
# launch shapes (build/bench/d1_walk).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/r03_f}
mkdir -p $OUT
for k in 12 20; do
  for p in "" "--periodic"; do
    LD_LIBRARY_PATH=build/var/bp timeout -k 10 120 build/bin/mpi_jacobi2d --ny=700 --nx=1900 0 47 --check --tblock --tsteps=$k \
      $p 2>&1 | grep -E "check" || { echo "bp check K=$k $p failed"; exit 1; }
  done
done
timeout -k 10 300 build/bench/d1_walk > $OUT/d1_walk.txt 2>&1 || { cat $OUT/d1_walk.txt; exit 1; }
cat $OUT/d1_walk.txt
B=build/bin/gmt_kernel_bench
for rep in 1 2; do
  for v in base bp ns; do
    lp=""; [ "$v" != base ] && lp=build/var/$v
    : > $OUT/$v.$rep.log
    for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" "--jacobi-n=8192 --iters=100"; do
      LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/$v.$rep.log 2>&1 || { cat $OUT/$v.$rep.log; exit 1; }
    done
    echo "$v: $(grep MLUPS $OUT/$v.$rep.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
  done
done
