#!/bin/bash
# Round 3: the oversubscribed multi-rank tests (IPC) and smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r03_c
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v --timeout 480 --timeout-method thread -m gpu tests/test_multirank_gpu.py \
  > $OUT/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error|PASS|FAIL" $OUT/pytest.log | tail -8
[ $rc = 0 ] || { tail -60 $OUT/pytest.log; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
