#!/bin/bash
# Round 4 (o): the host-staged exchange against its own bound.  The MPI leg
# alone (build/bin-host: the CPU backend, host buffers, the same MPI) vs
# mpi-host on the GPU (kernel-staged blocks, GMT_HOST_BLOCKS=1 default, vs
# packed faces, GMT_HOST_BLOCKS=0), and mpi_stencil2d_sycl 1024 1 at 2 ranks;
# 4 alternating repetitions; GMT_NUMA_BIND=1 (default: ranks on their GPU's
# socket) vs 0.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_o2}
mkdir -p $OUT
MPI=/opt/conda/bin/mpirun
: > $OUT/summary.txt
for rep in 1 2 3 4; do
  timeout -k 10 120 $MPI -np 2 build/bin-host/mpi_halo_bench 1048576 16777216 20 --transport=mpi-direct \
    > $OUT/mpi_only.$rep.log 2>&1 || { tail $OUT/mpi_only.$rep.log; exit 1; }
  echo "rep $rep MPI alone (host buffers):" >> $OUT/summary.txt; grep -E "^ +[0-9]+ +2 " $OUT/mpi_only.$rep.log >> $OUT/summary.txt
  for cfg in "1 1" "0 1" "1 0"; do
    set -- $cfg; hb=$1; nb=$2; t=b$hb.n$nb.$rep
    GMT_NUMA_BIND=$nb GMT_HOST_BLOCKS=$hb timeout -k 10 120 $MPI -np 2 build/bin/mpi_halo_bench 1048576 16777216 20 --transport=mpi-host \
      > $OUT/host_$t.log 2>&1 || { tail $OUT/host_$t.log; exit 1; }
    echo "rep $rep mpi-host GMT_HOST_BLOCKS=$hb GMT_NUMA_BIND=$nb:" >> $OUT/summary.txt; grep -E "^ +[0-9]+ +2 " $OUT/host_$t.log >> $OUT/summary.txt
    GMT_NUMA_BIND=$nb GMT_HOST_BLOCKS=$hb timeout -k 10 120 $MPI -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50 \
      > $OUT/sycl_$t.log 2>&1 || { tail $OUT/sycl_$t.log; exit 1; }
    echo "rep $rep sycl 1024 1 GMT_HOST_BLOCKS=$hb GMT_NUMA_BIND=$nb: $(grep 'exchange time' $OUT/sycl_$t.log | tr '\n' ' ')" >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
