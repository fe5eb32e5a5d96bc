#!/bin/bash
# Round-2 pass: full GPU test suite, smoke, bench.py (driver config + default),
# rocprofv3 kernel stats of the driver-config bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${1:-gpurun_out/full}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench_driver.json
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2>> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench_default.json
R=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/$OUT/prof.log 2>&1 || { tail -20 $R/$OUT/prof.log; exit 1; }
echo PROF_OK
