#!/bin/bash
# hygiene pass: production-only kernels + variant_bench; dim-1 derivative timing
set -o pipefail
mkdir -p gpurun_out/hyg
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/hyg/tests.log 2>&1 || { tail -40 gpurun_out/hyg/tests.log; exit 1; }
tail -2 gpurun_out/hyg/tests.log
timeout -k 10 300 build/bench/variant_bench > gpurun_out/hyg/variant_bench.log 2>&1; rc=$?
cat gpurun_out/hyg/variant_bench.log; [ $rc = 0 ] || exit 1
timeout -k 10 120 build/bin/gmt_kernel_bench --only=stencil --iters=20 --sustained=1 > gpurun_out/hyg/stencil.log 2>&1 && cat gpurun_out/hyg/stencil.log
