#!/bin/bash
# Round 3: whole GPU suite (incl. oversubscribed multi-rank IPC bench tests), smoke, driver bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r03_d
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v --timeout 480 --timeout-method thread -m gpu tests \
  > $OUT/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error" $OUT/pytest.log | tail -4
[ $rc = 0 ] || { grep -B5 -A40 "FAILURES" $OUT/pytest.log | head -80; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json
