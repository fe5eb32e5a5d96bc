#!/bin/bash
# host-staged transport (pipelined chunks) and IPC numbers, 2 ranks on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${1:-gpurun_out/xport}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
B=build/bin
run() { local t=$1 name=$2; shift 2; echo "=== $name: $*" >> $OUT/summary.txt; timeout -k 10 $t "$@" >> $OUT/summary.txt 2>&1 || { echo "FAILED $name rc=$?"; tail -20 $OUT/summary.txt; exit 1; }; }
: > $OUT/summary.txt
run 120 halo_host2 $M -np 2 $B/mpi_halo_bench 16 16777216 20 --transport=mpi-host
run 120 halo_ipc2 $M -np 2 $B/mpi_halo_bench 16 16777216 20 --transport=ipc
run 120 sycl_stage1 $M -np 2 $B/mpi_stencil2d_sycl 1024 1 50
run 120 sycl_stage0 $M -np 2 $B/mpi_stencil2d_sycl 1024 0 50
grep -E "^ +[0-9]+ +2 |exchange time|===" $OUT/summary.txt
