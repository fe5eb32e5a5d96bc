#!/bin/bash
# Round 6, final tree: the GPU suite, smoke, the driver-config bench three
# times, and a kernel-trace profile of one bench run (rocprofv3 --stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_final2
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.out 2> $OUT/bench_$i.err || { tail -30 $OUT/bench_$i.err; exit 1; }
  tail -1 $OUT/bench_$i.out > $OUT/bench_$i.json
  python3 -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('bench', d['value'], d.get('timed_pass_sclk_mhz'), d.get('timed_check_mismatches'), d.get('stencil_8192_MLUPS'), d.get('stencil_8192_check_mismatches'), d.get('daxpy_GBps'), d.get('halo_exchange_us'))"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_bench.out 2> $OUT/prof_bench.err || { tail -30 $OUT/prof_bench.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
echo R06FINAL2_OK
