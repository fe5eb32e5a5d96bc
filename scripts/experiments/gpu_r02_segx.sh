#!/bin/bash
# why are long segments slower?  rule path on/off (mask 0 / 15), seg 192..4096
set -o pipefail
mkdir -p gpurun_out/segx
for m in 0 15; do
timeout -k 10 300 build/bin/gmt_kernel_bench --only=tb --tb-k=20 --tb-nw=2 --tb-mask=$m \
  --tb-seg=192,384,768,1024,2048,4096 --jacobi-n=32768 --iters=6 --sustained=1 \
  > gpurun_out/segx/m$m.log 2>&1 && grep MLUPS gpurun_out/segx/m$m.log
done
