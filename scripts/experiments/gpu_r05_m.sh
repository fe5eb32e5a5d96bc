#!/bin/bash
# Round 5 (m): edge / boundary tiles round-robin over the XCDs
# (GMT_TB_SPECIAL_RR=1) x planner rule cost, Dirichlet domains; push ratio;
# per-workgroup timelines with RR; host-staged exchange (flat copies on a
# side stream, scatters on the caller's), ranks bound.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_m
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
    for rr in 0 1; do
      for c in 1.4 1.8; do
        echo "== rr$rr c$c $shp" >> $OUT/rates.log
        GMT_TB_SPECIAL_RR=$rr GMT_TB_RULE_COST=$c timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
    echo "== m15 $shp" >> $OUT/rates.log
    timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=15 $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
: > $OUT/kpush.log
for rr in 0 1; do
  for shp in "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
    echo "== rr$rr $shp" >> $OUT/kpush.log
    GMT_TB_SPECIAL_RR=$rr timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=15 --tb-push=1 $shp >> $OUT/kpush.log 2>&1 || { tail -20 $OUT/kpush.log; exit 1; }
  done
done
grep -E "^==|ratio" $OUT/kpush.log
for cfg in "n32768_m0:--jacobi-n=32768 --tb-mask=0 --iters=30" "n8192_m0:--jacobi-n=8192 --tb-mask=0 --iters=100" \
           "r8k16k_m0:--jacobi-ny=8192 --jacobi-nx=16384 --tb-mask=0 --iters=60" \
           "r8k16k_push:--jacobi-ny=8192 --jacobi-nx=16384 --tb-mask=15 --tb-push=1 --iters=60"; do
  name=${cfg%%:*}; opts=${cfg#*:}
  GMT_TB_SPECIAL_RR=1 LD_LIBRARY_PATH=$R/build/var/wgt GMT_TB_WG_TRACE_FILE=$OUT/wg_rr_$name.txt GMT_TB_WG_TRACE_LAUNCH=25 \
    timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 $opts > $OUT/kb_$name.log 2>&1 || { tail -20 $OUT/kb_$name.log; exit 1; }
done
M=/opt/conda/bin/mpirun
for rep in 1 2 3; do
  mkdir -p $OUT/halo_$rep $OUT/sycl_$rep
  GMT_HOST_TRACE=$OUT/halo_$rep timeout -k 10 120 $M -np 2 -bind-to core build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_$rep.txt 2>&1 || { tail $OUT/halo_$rep.txt; exit 1; }
  GMT_HOST_TRACE=$OUT/sycl_$rep timeout -k 10 120 $M -np 2 -bind-to core build/bin/mpi_stencil2d_sycl 1024 1 > $OUT/sycl_$rep.txt 2>&1 || { tail $OUT/sycl_$rep.txt; exit 1; }
  echo "rep $rep: mpi-host $(grep -E '^ *8388608' $OUT/halo_$rep.txt | head -1) | sycl $(grep 'exchange time' $OUT/sycl_$rep.txt | head -1)"
done
echo R05M_OK
