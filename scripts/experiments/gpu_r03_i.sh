#!/bin/bash
# Round 3: after 3/4-length W/E signalling segments and the register-window
# dim-1 derivative: whole GPU suite, smoke, driver bench, derivative rate at
# the reference's dim-1 shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r03_i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A40 "FAILURES" $OUT/pytest.log | head -80; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -2 $OUT/smoke.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json &&
timeout -k 10 120 build/bin/gmt_kernel_bench --only=stencil > $OUT/deriv.txt 2>&1; tail -12 $OUT/deriv.txt
