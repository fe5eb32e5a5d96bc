#!/bin/bash
# memory-path experiments on the K=4/8/12 passes (timing only)
set -o pipefail
mkdir -p gpurun_out/r2n
B=build/bin/gmt_kernel_bench
for v in base st0 dmant p6; do
  echo "== $v"
  LD_LIBRARY_PATH=$PWD/build/exp/$v timeout -k 10 200 $B --only=tb --iters=7 --tb-k=4,8,12 --tb-nw=4 --tb-seg=0,64,96 > gpurun_out/r2n/$v.log 2>&1 || { tail -3 gpurun_out/r2n/$v.log; exit 1; }
  grep " ms" gpurun_out/r2n/$v.log | awk '{print $3, $4, $5, $8, $9}'
done
