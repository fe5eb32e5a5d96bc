#!/bin/bash
# halo latency (blocking and stream-ordered) per transport, then the strong-scaling shares
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/lat
M=/opt/conda/bin/mpirun
timeout -k 10 120 $M -np 2 build/bin/mpi_halo_bench 16 16777216 50 --transport=ipc > gpurun_out/lat/ipc2.log 2>&1 || exit 1
timeout -k 10 120 $M -np 1 build/bin/mpi_halo_bench 16 16777216 50 --transport=rccl > gpurun_out/lat/rccl1.log 2>&1 || exit 1
timeout -k 10 120 $M -np 2 build/bin/mpi_halo_bench 16 16777216 20 --transport=mpi-host > gpurun_out/lat/host2.log 2>&1 || exit 1
head -8 gpurun_out/lat/ipc2.log; head -8 gpurun_out/lat/rccl1.log | tail -6
./scripts/gpu_r02_shares.sh
