#!/bin/bash
# Round 4 (g): after the GPU suite passed (r04_f: 776 tests),
#  (1) wide K = 20 kernel (build/ab_wide, opt-in) and its diagnostics (P = 9, no step
#      barrier, FLOW counters) vs production (narrow, = round 3),
#  (2) the strong-scaling shares, serial vs band-first with column bands,
#  (3) mpi-host: faces staged in place vs packed (GMT_HOST_BLOCKS=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_g}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
B=$R/build/bin/gmt_kernel_bench
# the FLOW variant (LDS progress counters instead of step barriers): bitwise first
for p in "" "--periodic"; do
  LD_LIBRARY_PATH=$R/build/ab_flow timeout -k 10 120 build/bin/mpi_jacobi2d --ny=700 --nx=1900 0 47 --check --tblock --tsteps=20 $p 2>&1 | grep -E "vs serial" | tee -a $OUT/flow_check.txt
done
for rep in 1 2; do
  for v in new wide flow nobar p9; do
    lp=""; [ "$v" != new ] && lp=$R/build/ab_$v
    : > $OUT/$v.$rep.log
    for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100"; do
      LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/$v.$rep.log 2>&1 || { cat $OUT/$v.$rep.log; exit 1; }
    done
    echo "$v: $(grep MLUPS $OUT/$v.$rep.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
  done
done
: > $OUT/shares.txt
for rep in 1 2; do
  for cfg in "32768 32768" "16384 32768" "16384 16384" "8192 16384" "16384 8192"; do
    set -- $cfg
    for mode in "--no-overlap" "--overlap"; do
      timeout -k 10 200 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 --graph \
        --periodic --transport=rccl $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
      echo "rep=$rep ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log)" | tee -a $OUT/shares.txt
    done
  done
done
run() { local t=$1 name=$2; shift 2; echo "=== $name: $*" >> $OUT/xport.txt; timeout -k 10 $t "$@" >> $OUT/xport.txt 2>&1 || { echo "FAILED $name rc=$?"; tail -20 $OUT/xport.txt; exit 1; }; }
: > $OUT/xport.txt
for rep in 1 2; do
  run 120 sycl_blocks_$rep $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50
  GMT_HOST_BLOCKS=0 run 120 sycl_packed_$rep $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50
  run 120 halo_blocks_$rep $M -np 2 build/bin/mpi_halo_bench 65536 16777216 20 --transport=mpi-host
  GMT_HOST_BLOCKS=0 run 120 halo_packed_$rep $M -np 2 build/bin/mpi_halo_bench 65536 16777216 20 --transport=mpi-host
done
grep -E "^ +[0-9]+ +2 |exchange time|===" $OUT/xport.txt
