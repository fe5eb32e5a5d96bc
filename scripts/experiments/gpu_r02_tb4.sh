#!/bin/bash
# 3-column / two-stage temporal-blocking kernel: bitwise tests, then pass
# costs per K at 32768^2 and 8192^2 (sustained: back-to-back launches).
set -o pipefail
mkdir -p gpurun_out/tb4
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_jacobi_tb_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/tb4/tests.log 2>&1 || { tail -30 gpurun_out/tb4/tests.log; exit 1; }
tail -3 gpurun_out/tb4/tests.log
KS=1,2,3,4,5,6,7,8,9,10,12,14,16,18,20,22,24
timeout -k 10 300 build/bin/gmt_kernel_bench --only=tb --tb-k=$KS --jacobi-n=32768 --iters=10 --sustained=1 \
  > gpurun_out/tb4/costs_32768.log 2>&1 && cat gpurun_out/tb4/costs_32768.log | grep MLUPS
timeout -k 10 300 build/bin/gmt_kernel_bench --only=tb --tb-k=$KS --jacobi-n=8192 --iters=50 --sustained=1 \
  > gpurun_out/tb4/costs_8192.log 2>&1 && cat gpurun_out/tb4/costs_8192.log | grep MLUPS
