#!/bin/bash
# 4-column kernel after the per-K translation-unit split: bitwise tests,
# counters of the K = 12 / 20 passes, strong-scaling shares
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tb4d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_jacobi_tb_gpu.py > $OUT/pytest_tb.log 2>&1 || { tail -40 $OUT/pytest_tb.log; exit 1; }
tail -1 $OUT/pytest_tb.log
scripts/gpu_r02_pmc.sh $OUT/pmc --only=hot --hot-k=12,20 --iters=3 || exit 1
OUT=$OUT/shares bash scripts/gpu_r02_shares.sh > $OUT/shares.txt 2>&1 || { tail -20 $OUT/shares.txt; exit 1; }
cat $OUT/shares.txt
