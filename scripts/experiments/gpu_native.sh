#!/bin/bash
# Native-app validation on one MI355X (run through gpurun).  Every GPU step
# has its own time limit and the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/native
mkdir -p $OUT
: > $OUT/results.jsonl
MPIRUN=/opt/conda/bin/mpirun
B=build/bin
n=0
run() {  # run <seconds> <name> <cmd...>
  local t=$1 name=$2; shift 2
  n=$((n+1))
  echo "=== [$n] $name: $*" | tee -a $OUT/summary.txt
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -n 25 $OUT/$name.log >> $OUT/summary.txt
  if [ $rc -ne 0 ]; then
    echo "FAILED rc=$rc at $name" | tee -a $OUT/summary.txt
    tail -n 40 $OUT/$name.log
    exit $rc
  fi
}
J="--json=$OUT/results.jsonl"
run 60  daxpy            $B/daxpy
run 120 daxpy_2e28       $B/daxpy --n=268435456 --iters=30 $J
run 120 daxpy_2e28_rb    $B/daxpy --n=268435456 --iters=30 --rocblas $J
run 60  daxpy_nvtx       $B/daxpy_nvtx --print=0
run 60  mpi_daxpy        $MPIRUN -np 1 $B/mpi_daxpy
run 60  mpi_daxpy_gt     $MPIRUN -np 2 $B/mpi_daxpy_gt
run 60  mpienv           env MEMORY_PER_CORE=2048 $MPIRUN -np 2 $B/mpienv
run 120 jacobi_check1    $MPIRUN -np 1 $B/mpi_jacobi2d 515 30 --check --warmup=3
run 120 jacobi_check_p   $MPIRUN -np 1 $B/mpi_jacobi2d 515 30 --check --periodic --graph --warmup=3
run 120 jacobi_check_rccl $MPIRUN -np 1 $B/mpi_jacobi2d 515 30 --check --periodic --graph --transport=rccl --warmup=3
run 120 jacobi_check_ipc2 $MPIRUN -np 2 $B/mpi_jacobi2d 515 30 --check --transport=ipc --warmup=3
run 120 jacobi_check_host4 $MPIRUN -np 4 $B/mpi_jacobi2d 300 20 --check --dims=2x2 --transport=mpi-host --warmup=3
run 180 jacobi_8192      $MPIRUN -np 1 $B/mpi_jacobi2d 8192 200 $J
run 240 jacobi_32768     $MPIRUN -np 1 $B/mpi_jacobi2d 32768 50 $J
run 240 jacobi_32768_p   $MPIRUN -np 1 $B/mpi_jacobi2d 32768 50 --periodic --graph --transport=rccl --halo-iters=50 $J
run 240 jacobi_8192_prg  $MPIRUN -np 1 $B/mpi_jacobi2d 8192 200 --periodic --graph --transport=rccl --halo-iters=50 $J
run 120 halo_rccl1       $MPIRUN -np 1 $B/mpi_halo_bench 16 67108864 30 --transport=rccl $J
run 120 halo_ipc2        $MPIRUN -np 2 $B/mpi_halo_bench 16 67108864 30 --transport=ipc $J
run 120 halo_host2       $MPIRUN -np 2 $B/mpi_halo_bench 16 16777216 20 --transport=mpi-host $J
run 60  stencil1d        $MPIRUN -np 2 $B/mpi_stencil_gt 32 --iters=100 $J
run 300 stencil2d_gt1    $MPIRUN -np 1 $B/mpi_stencil2d_gt 1024 50 $J
run 300 stencil2d_gt2    $MPIRUN -np 2 $B/mpi_stencil2d_gt 1024 30 --no-managed $J
run 60  buf_view         $B/mpi_stencil2d_sycl --test-buf-view=64
run 120 stencil2d_sycl   $MPIRUN -np 2 $B/mpi_stencil2d_sycl 1024 0 50 $J
run 120 stencil2d_sycl_h $MPIRUN -np 2 $B/mpi_stencil2d_sycl 1024 1 50 $J
run 120 stencil2d_oo     $MPIRUN -np 2 $B/mpi_stencil2d_sycl_oo 8 0 100 $J
run 120 daxpy_nvtx_man   $MPIRUN -np 2 $B/mpi_daxpy_nvtx_managed --iters=10 $J
run 120 daxpy_nvtx_unm   $MPIRUN -np 2 $B/mpi_daxpy_nvtx_unmanaged --iters=10 $J
run 180 gather_host      $MPIRUN -np 2 $B/mpigatherinplace --n=33554432 $J
run 180 gather_dev       $MPIRUN -np 2 $B/mpigatherinplace --n=33554432 --device $J
echo "ALL OK" | tee -a $OUT/summary.txt
