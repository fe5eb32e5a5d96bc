#!/bin/bash
# tb kernel numerics (all failures listed) + counters of old vs new kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${1:-gpurun_out/tbpmc}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_jacobi_tb_gpu.py -q --maxfail=40 --timeout 120 --timeout-method thread \
  > "$OUT/pytest_tb.log" 2>&1
rc=$?
grep -E "passed|failed" "$OUT/pytest_tb.log" | tail -3
grep FAILED "$OUT/pytest_tb.log" | head -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
scripts/gpu_r02_pmc.sh "$OUT/pmc" --only=hot,tb --hot-k=12 --tb-k=12 --tb-nw=1,4 --tb-p=5 --iters=2 || exit 1
exit 0
