#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/probe
mkdir -p $OUT
timeout -k 10 60 build/bench/buffer_oob > $OUT/oob.log 2>&1 || { cat $OUT/oob.log; exit 1; }
cat $OUT/oob.log
timeout -k 10 400 build/bin/gmt_kernel_bench --iters=10 --only=jacobi --sections=pipe --jacobi-n=32768 > $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
grep -E "pipe" $OUT/kb.log
