#!/bin/bash
# segment length x strips-per-workgroup sweep of the 3-column kernel (sustained)
set -o pipefail
mkdir -p gpurun_out/tb4
timeout -k 10 400 build/bin/gmt_kernel_bench --only=tb --tb-k=12,16,20 --tb-nw=1,2,4 \
  --tb-seg=192,256,384,512,768,1024 --jacobi-n=32768 --iters=8 --sustained=1 \
  > gpurun_out/tb4/seg_32768.log 2>&1 && grep MLUPS gpurun_out/tb4/seg_32768.log
timeout -k 10 300 build/bin/gmt_kernel_bench --only=tb --tb-k=2,8,10,12,14 --tb-nw=1,2,4,8 \
  --tb-seg=48,64,96,128,192,256 --jacobi-n=8192 --iters=40 --sustained=1 \
  > gpurun_out/tb4/seg_8192.log 2>&1 && grep MLUPS gpurun_out/tb4/seg_8192.log
