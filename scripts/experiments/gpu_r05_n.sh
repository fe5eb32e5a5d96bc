#!/bin/bash
# Round 5 (n): same-box A/B of the host-staged receive leg (flat chunks' H2D
# copies on a side stream vs the caller's stream), ranks bound to cores,
# alternating with MPI alone; the reference's stage_host exchange.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_n
mkdir -p $OUT
M=/opt/conda/bin/mpirun
for rep in 1 2 3 4; do
  timeout -k 10 120 $M -np 2 -bind-to core build/bin-host/mpi_halo_bench 8388608 8388608 30 --transport=mpi-direct > $OUT/alone_$rep.txt 2>&1 || { tail $OUT/alone_$rep.txt; exit 1; }
  for rs in 1 0; do
    mkdir -p $OUT/halo_rs${rs}_$rep
    GMT_HOST_RECV_STREAM=$rs GMT_HOST_TRACE=$OUT/halo_rs${rs}_$rep timeout -k 10 120 $M -np 2 -bind-to core build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_rs${rs}_$rep.txt 2>&1 || { tail $OUT/halo_rs${rs}_$rep.txt; exit 1; }
  done
  timeout -k 10 120 $M -np 2 -bind-to core build/bin/mpi_stencil2d_sycl 1024 1 > $OUT/sycl_$rep.txt 2>&1 || { tail $OUT/sycl_$rep.txt; exit 1; }
  echo "rep $rep: alone $(grep -E '^ *8388608' $OUT/alone_$rep.txt | head -1) | side $(grep -E '^ *8388608' $OUT/halo_rs1_$rep.txt | head -1) | caller $(grep -E '^ *8388608' $OUT/halo_rs0_$rep.txt | head -1) | sycl $(grep 'exchange time' $OUT/sycl_$rep.txt | head -1)"
done
echo R05N_OK
