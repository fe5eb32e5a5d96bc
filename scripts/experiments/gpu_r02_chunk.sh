#!/bin/bash
# mpi-host pipeline chunk size sweep (2 ranks, one GPU)
set -o pipefail
M=/opt/conda/bin/mpirun
mkdir -p gpurun_out/chunk
for kb in 128 512 1024 4096 65536; do
  timeout -k 10 120 $M -np 2 -env GMT_HOST_CHUNK_KB $kb build/bin/mpi_halo_bench 1048576 16777216 20 --transport=mpi-host > gpurun_out/chunk/c$kb.log 2>&1 || exit 1
  echo "chunk ${kb}KB: $(grep -E '^ +[0-9]+ +2 ' gpurun_out/chunk/c$kb.log | tr -s ' ' | cut -d' ' -f2,4,6 | tr '\n' '|')"
  timeout -k 10 120 $M -np 2 -env GMT_HOST_CHUNK_KB $kb build/bin/mpi_stencil2d_sycl 1024 1 50 > gpurun_out/chunk/s$kb.log 2>&1 || exit 1
  echo "   sycl stage1: $(grep 'exchange time' gpurun_out/chunk/s$kb.log | head -1)"
done
