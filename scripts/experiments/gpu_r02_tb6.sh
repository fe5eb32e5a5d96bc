#!/bin/bash
# boundary-group segments: tests, costs at 32768/8192 (sustained), shares
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/tb6
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_jacobi_tb_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/tb6/tests.log 2>&1 || { tail -30 gpurun_out/tb6/tests.log; exit 1; }
tail -1 gpurun_out/tb6/tests.log
KS=1,2,3,4,5,6,7,8,9,10,12,14,16,18,20,22,24
timeout -k 10 300 build/bin/gmt_kernel_bench --only=tb --tb-k=$KS --jacobi-n=32768 --iters=8 --sustained=1 \
  > gpurun_out/tb6/costs_32768.log 2>&1 && grep MLUPS gpurun_out/tb6/costs_32768.log
timeout -k 10 300 build/bin/gmt_kernel_bench --only=tb --tb-k=$KS --jacobi-n=8192 --iters=40 --sustained=1 \
  > gpurun_out/tb6/costs_8192.log 2>&1 && grep MLUPS gpurun_out/tb6/costs_8192.log
