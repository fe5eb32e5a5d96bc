#!/bin/bash
# variant_bench timing + production stencil timing
set -o pipefail
mkdir -p gpurun_out/hyg
timeout -k 10 300 build/bench/variant_bench > gpurun_out/hyg/variant_bench.log 2>&1; rc=$?
cat gpurun_out/hyg/variant_bench.log; [ $rc = 0 ] || exit 1
timeout -k 10 120 build/bin/gmt_kernel_bench --only=stencil --iters=20 --sustained=1 > gpurun_out/hyg/stencil.log 2>&1 && cat gpurun_out/hyg/stencil.log
