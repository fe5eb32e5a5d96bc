#!/bin/bash
# Round 3 GPU pass: driver-config bench (random init, calibrated plan), the
# whole GPU suite (incl. the oversubscribed multi-rank bench tests), smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r03_b
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 1000 python -u -m pytest -x -v --timeout 480 --timeout-method thread -m gpu tests \
  > $OUT/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error" $OUT/pytest.log | tail -5
[ $rc = 0 ] || { tail -60 $OUT/pytest.log; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
