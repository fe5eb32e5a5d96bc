#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2o
B=build/bin/gmt_kernel_bench
for v in p6b p9; do
  echo "== $v"
  LD_LIBRARY_PATH=$PWD/build/exp/$v timeout -k 10 200 $B --only=tb --iters=7 --tb-k=2,4,6,8,10 --tb-nw=4 > gpurun_out/r2o/$v.log 2>&1 || { tail -3 gpurun_out/r2o/$v.log; exit 1; }
  grep " ms" gpurun_out/r2o/$v.log | awk '{print $3, $4, $5, $8, $9}'
  LD_LIBRARY_PATH=$PWD/build/exp/$v timeout -k 10 200 $B --only=tb --iters=15 --jacobi-n=8192 --tb-k=8,10 --tb-nw=4 > gpurun_out/r2o/${v}_8192.log 2>&1 || { tail -3 gpurun_out/r2o/${v}_8192.log; exit 1; }
  grep " ms" gpurun_out/r2o/${v}_8192.log | awk '{print $3, $4, $5, $8, $9}'
done
