#!/bin/bash
# Round 3: host-staged transport, kernel-driven D2H staging (GMT_HOST_STAGE=kernel,
# default) vs the round-2 SDMA chunks (sdma), 2 ranks on one GPU; the
# reference's stage_host exchange; IPC latency after the table-driven kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${1:-gpurun_out/r03_xport}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
run() { local t=$1 name=$2; shift 2; echo "=== $name: $*" >> $OUT/summary.txt; timeout -k 10 $t "$@" >> $OUT/summary.txt 2>&1 || { echo "FAILED $name rc=$?"; tail -20 $OUT/summary.txt; exit 1; }; }
: > $OUT/summary.txt
for rep in 1 2; do
GMT_HOST_STAGE=kernel run 120 halo_host_kernel_$rep $M -np 2 build/bin/mpi_halo_bench 65536 16777216 20 --transport=mpi-host
GMT_HOST_STAGE=sdma run 120 halo_host_sdma_$rep $M -np 2 build/bin/mpi_halo_bench 65536 16777216 20 --transport=mpi-host
GMT_HOST_STAGE=kernel run 120 sycl_stage1_kernel_$rep $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50
GMT_HOST_STAGE=sdma run 120 sycl_stage1_sdma_$rep $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50
done
run 120 halo_ipc2 $M -np 2 build/bin/mpi_halo_bench 16 1024 200 --transport=ipc
run 120 host_mpi_ceiling $M -np 2 build/bin-host/mpi_halo_bench 65536 16777216 20 --transport=mpi-direct
grep -E "^ +[0-9]+ +2 |exchange time|===" $OUT/summary.txt
