#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep2
timeout -k 10 400 build/bench/stream_sweep 268435456 32768 2 > gpurun_out/sweep2/sweep2.log 2>&1 || { cat gpurun_out/sweep2/sweep2.log; exit 1; }
cat gpurun_out/sweep2/sweep2.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sweep2/prof -o kb -- $GRAFT_REPO_ROOT/build/bin/gmt_kernel_bench --iters=5 --only=daxpy > $GRAFT_REPO_ROOT/gpurun_out/sweep2/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/sweep2/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/sweep2/prof -name "*.csv" | head
