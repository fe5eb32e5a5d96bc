#!/bin/bash
# Round 6 (d): rank pinning of the host-staged exchange, four modes
# alternating: pinned before MPI_Init near the GPU (default), pinned before
# MPI_Init from the start of the allowed set (GMT_PIN_NEAR=0), unpinned
# (GMT_PIN=0), and mpirun -bind-to core (round 5's fix) — 2 ranks, 8 MiB,
# mpi_halo_bench and the reference's stage_host exchange (sycl 1024 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_d
mkdir -p $OUT
M=/opt/conda/bin/mpirun
: > $OUT/pin_modes.txt
nproc > $OUT/machine.txt; cat /sys/fs/cgroup/cpuset.cpus.effective >> $OUT/machine.txt 2>/dev/null; python3 -c "import os; print(sorted(os.sched_getaffinity(0))[:8], len(os.sched_getaffinity(0)))" >> $OUT/machine.txt
for rep in 1 2 3 4; do
  for mode in near start none bind; do
    env=""; b=""
    case $mode in start) env="GMT_PIN_NEAR=0";; none) env="GMT_PIN=0";; bind) env="GMT_PIN=0"; b="-bind-to core";; esac
    env $env timeout -k 10 120 $M $b -np 2 build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_${mode}_$rep.txt 2>&1 || { tail $OUT/halo_${mode}_$rep.txt; exit 1; }
    env $env timeout -k 10 120 $M $b -np 2 build/bin/mpi_stencil2d_sycl 1024 1 > $OUT/sycl_${mode}_$rep.txt 2>&1 || { tail $OUT/sycl_${mode}_$rep.txt; exit 1; }
    echo "rep $rep $mode: $(grep 'pinned cpu' $OUT/halo_${mode}_$rep.txt) | $(grep -E '^ *8388608' $OUT/halo_${mode}_$rep.txt | head -1) | sycl $(grep 'exchange time' $OUT/sycl_${mode}_$rep.txt | tr '\n' ' ')" | tee -a $OUT/pin_modes.txt
  done
done
cat $OUT/machine.txt
echo R06D_OK
