#!/bin/bash
# Kernel-variant A/B sweep + numerics on one MI355X (through gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/kern
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 build/bin/gmt_kernel_bench --iters=20 --json=$OUT/kb.jsonl > $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
cat $OUT/kb.log
timeout -k 10 300 build/bin/gmt_kernel_bench --iters=20 --jacobi-n=8192 --only=jacobi > $OUT/kb8192.log 2>&1 || { cat $OUT/kb8192.log; exit 1; }
cat $OUT/kb8192.log
