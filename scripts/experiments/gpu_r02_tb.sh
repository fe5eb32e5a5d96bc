#!/bin/bash
# Round 2: numerics of the temporal-blocking kernel (jacobi5tb.hip), then its
# timing sweep at 32768^2 and 8192^2 next to the round-1 pipelined kernel.
# Usage: scripts/gpu_r02_tb.sh OUTDIR [kernel-bench tb args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${1:-gpurun_out/tb}
shift
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_jacobi_tb_gpu.py -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest_tb.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_tb.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
B=build/bin/gmt_kernel_bench
timeout -k 10 300 $B --only=hot,tb --iters=5 "$@" > "$OUT/kb_32768.log" 2>&1 || { tail -20 "$OUT/kb_32768.log"; exit 1; }
cat "$OUT/kb_32768.log"
timeout -k 10 300 $B --only=hot,tb --iters=10 --jacobi-n=8192 "$@" > "$OUT/kb_8192.log" 2>&1 || { tail -20 "$OUT/kb_8192.log"; exit 1; }
grep MLUPS "$OUT/kb_8192.log"
exit $rc
