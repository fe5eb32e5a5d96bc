#!/bin/bash
# Round 3: the multi-rank GPU tests (2, 4 and 8 ranks sharing cuda:0 over IPC, peer-hang fault injection).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r03_mr
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 480 --timeout-method thread -m gpu tests/test_multirank_gpu.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -8 $OUT/pytest.log
