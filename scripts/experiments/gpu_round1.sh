#!/bin/bash
# First GPU validation: kernel numerics, smoke, short bench, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo "bench failed"; tail -30 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
for v in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --variant $v --skip-extras > gpurun_out/bench_v$v.json 2>>gpurun_out/bench1.err || exit 1
  cat gpurun_out/bench_v$v.json
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof1.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof1 -name "*stats*" | head
