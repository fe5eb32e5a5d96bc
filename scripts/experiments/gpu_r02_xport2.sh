#!/bin/bash
# transport ceilings on the 1-GPU box, 2 ranks: pure host MPI (CPU backend,
# host memory: the ceiling of any host-staged path), host-staged from device
# memory, stream-ordered IPC latency, and the reference's stage_host exchange
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${1:-gpurun_out/xport2}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
run() { local t=$1 name=$2; shift 2; echo "=== $name: $*" >> $OUT/summary.txt; timeout -k 10 $t "$@" >> $OUT/summary.txt 2>&1 || { echo "FAILED $name rc=$?"; tail -20 $OUT/summary.txt; exit 1; }; }
: > $OUT/summary.txt
run 120 host_mpi_ceiling $M -np 2 build/bin-host/mpi_halo_bench 65536 16777216 20 --transport=mpi-direct
run 120 halo_host2 $M -np 2 build/bin/mpi_halo_bench 65536 16777216 20 --transport=mpi-host
run 120 halo_ipc2 $M -np 2 build/bin/mpi_halo_bench 16 1024 200 --transport=ipc
run 120 sycl_stage1 $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50
grep -E "^ +[0-9]+ +2 |exchange time|===" $OUT/summary.txt
