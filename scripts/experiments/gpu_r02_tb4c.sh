#!/bin/bash
# 4-column / skew-1 temporal-blocking kernel: bitwise tests, then the driver
# bench config, kernel resources and a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tb4c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_jacobi_tb_gpu.py > $OUT/pytest_tb.log 2>&1 || { tail -40 $OUT/pytest_tb.log; exit 1; }
tail -1 $OUT/pytest_tb.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench_driver.json
timeout -k 10 300 build/bin/gmt_kernel_bench --only=tb --iters=30 --sustained=1 --tb-k=20 --tb-nw=2 --tb-mask=0 --jacobi-n=32768 > $OUT/kb20.log 2>&1 || { cat $OUT/kb20.log; exit 1; }
grep -E "MLUPS|vgpr|VGPR" $OUT/kb20.log | head
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --skip-extras > $R/$OUT/prof.log 2>&1 || { tail -20 $R/$OUT/prof.log; exit 1; }
echo PROF_OK
