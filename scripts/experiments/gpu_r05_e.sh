#!/bin/bash
# Round 5 (e): the host-staged exchange's slow mode, traced.  Six alternating
# repetitions of (a) MPI alone on host buffers (the CPU backend's
# mpi-direct: the same MPICH, the same box) and (b) the mpi-host exchange at
# 8 MiB, and (c) the reference's stage_host benchmark (mpi_stencil2d_sycl
# 1024 1), 2 ranks sharing the GPU; every mpi-host exchange's host-side phases
# are written by GMT_HOST_TRACE (csrc/comm/transport_mpi.cpp).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r05_e}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
for rep in 1 2 3 4 5 6; do
  timeout -k 10 120 $M -np 2 build/bin-host/mpi_halo_bench 8388608 8388608 30 --transport=mpi-direct > $OUT/mpi_alone_$rep.txt 2>&1 || { tail $OUT/mpi_alone_$rep.txt; exit 1; }
  mkdir -p $OUT/halo_$rep
  GMT_HOST_TRACE=$OUT/halo_$rep timeout -k 10 120 $M -np 2 build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_$rep.txt 2>&1 || { tail $OUT/halo_$rep.txt; exit 1; }
  mkdir -p $OUT/sycl_$rep
  GMT_HOST_TRACE=$OUT/sycl_$rep timeout -k 10 120 $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 > $OUT/sycl_$rep.txt 2>&1 || { tail $OUT/sycl_$rep.txt; exit 1; }
  echo "rep $rep: alone $(grep -E '^ *8388608' $OUT/mpi_alone_$rep.txt | head -1) | mpi-host $(grep -E '^ *8388608' $OUT/halo_$rep.txt | head -1) | sycl $(grep 'exchange time' $OUT/sycl_$rep.txt | head -1)"
done
# the README's 16-B stream-ordered IPC latency, re-measured (2 ranks, 1 GPU)
for rep in 1 2 3; do
  timeout -k 10 120 $M -np 2 build/bin/mpi_halo_bench 16 4096 300 --transport=ipc > $OUT/ipc16_$rep.txt 2>&1 || { tail $OUT/ipc16_$rep.txt; exit 1; }
done
head -30 $OUT/ipc16_1.txt
echo R05E_OK
