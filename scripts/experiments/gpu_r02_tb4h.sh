#!/bin/bash
# kernel variant check: bitwise tests of the tb kernel, sustained K = 12/16/20
# at 32768^2 and the N = 8 share, driver bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tb4h}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_jacobi_tb_gpu.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=build/bin/gmt_kernel_bench
timeout -k 10 200 $B --only=tb --sustained=1 --iters=20 --tb-k=12,16,20 --tb-mask=0 --jacobi-n=32768 > $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
timeout -k 10 200 $B --only=tb --sustained=1 --iters=100 --tb-k=20 --tb-mask=0 --jacobi-ny=8192 --jacobi-nx=16384 >> $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
grep MLUPS $OUT/kb.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-extras > $OUT/bench_driver.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench_driver.json
