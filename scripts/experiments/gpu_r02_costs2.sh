#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${1:-gpurun_out/costs2}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_jacobi_tb_gpu.py -q -x --timeout 120 --timeout-method thread > "$OUT/pytest_tb.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_tb.log"
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
B=build/bin/gmt_kernel_bench
timeout -k 10 300 $B --only=tb --iters=7 --tb-k=2,4,6,8,10,12,14,16 --tb-nw=4 > "$OUT/kb_32768.log" 2>&1 || { tail -5 "$OUT/kb_32768.log"; exit 1; }
grep " ms" "$OUT/kb_32768.log"
timeout -k 10 300 $B --only=tb --iters=15 --jacobi-n=8192 --tb-k=8,10,12,14 --tb-nw=4 > "$OUT/kb_8192.log" 2>&1 || { tail -5 "$OUT/kb_8192.log"; exit 1; }
grep " ms" "$OUT/kb_8192.log"
