#!/bin/bash
# Round 5 (o): full GPU suite, smoke, driver-config bench; random vs analytic
# field data on the K = 20 pass (power / switching A/B).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_o
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out > $OUT/bench.json; cat $OUT/bench.json
timeout -k 10 300 python -u scripts/experiments/init_ab.py 8192 1000 > $OUT/init_ab_8192.log 2>&1 || { tail -20 $OUT/init_ab_8192.log; exit 1; }
cat $OUT/init_ab_8192.log
timeout -k 10 300 python -u scripts/experiments/init_ab.py 32768 60 > $OUT/init_ab_32768.log 2>&1 || { tail -20 $OUT/init_ab_32768.log; exit 1; }
cat $OUT/init_ab_32768.log
echo R05O_OK
