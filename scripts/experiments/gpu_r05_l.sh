#!/bin/bash
# Round 5 (l): per-workgroup timelines of the K = 20 pass (build/var/wgt:
# GMT_TB_WG_TRACE=1) — rule-path and push-body workgroup durations, per-XCD
# finish times — on the headline and share domains; then the host-staged
# exchange with the receive leg back on the caller's stream, ranks bound.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_l
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
for cfg in "n32768_m0:--jacobi-n=32768 --tb-mask=0 --iters=30" "n32768_m15:--jacobi-n=32768 --tb-mask=15 --iters=30" \
           "n8192_m0:--jacobi-n=8192 --tb-mask=0 --iters=100" "n8192_m15:--jacobi-n=8192 --tb-mask=15 --iters=100" \
           "r8k16k_m0:--jacobi-ny=8192 --jacobi-nx=16384 --tb-mask=0 --iters=60" \
           "r8k16k_push:--jacobi-ny=8192 --jacobi-nx=16384 --tb-mask=15 --tb-push=1 --iters=60" \
           "r16k8k_push:--jacobi-ny=16384 --jacobi-nx=8192 --tb-mask=15 --tb-push=1 --iters=60"; do
  name=${cfg%%:*}; opts=${cfg#*:}
  LD_LIBRARY_PATH=$R/build/var/wgt GMT_TB_WG_TRACE_FILE=$OUT/wg_$name.txt GMT_TB_WG_TRACE_LAUNCH=25 \
    timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 $opts > $OUT/kb_$name.log 2>&1 || { tail -20 $OUT/kb_$name.log; exit 1; }
  grep -E "MLUPS|ratio" $OUT/kb_$name.log | head -3
done
ls $OUT
M=/opt/conda/bin/mpirun
for rep in 1 2 3; do
  mkdir -p $OUT/halo_$rep
  GMT_HOST_TRACE=$OUT/halo_$rep timeout -k 10 120 $M -np 2 -bind-to core build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_$rep.txt 2>&1 || { tail $OUT/halo_$rep.txt; exit 1; }
  mkdir -p $OUT/sycl_$rep
  GMT_HOST_TRACE=$OUT/sycl_$rep timeout -k 10 120 $M -np 2 -bind-to core build/bin/mpi_stencil2d_sycl 1024 1 > $OUT/sycl_$rep.txt 2>&1 || { tail $OUT/sycl_$rep.txt; exit 1; }
  echo "rep $rep: mpi-host $(grep -E '^ *8388608' $OUT/halo_$rep.txt | head -1) | sycl $(grep 'exchange time' $OUT/sycl_$rep.txt | head -1)"
done
echo R05L_OK
