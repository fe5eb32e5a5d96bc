#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/x2b
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "jacobi5x2" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 build/bin/gmt_kernel_bench --iters=20 --only=jacobi --jacobi-n=8192 > $OUT/kb8k.log 2>&1 || { cat $OUT/kb8k.log; exit 1; }
grep x2 $OUT/kb8k.log
timeout -k 10 300 build/bin/gmt_kernel_bench --iters=10 --only=jacobi --jacobi-n=32768 > $OUT/kb32k.log 2>&1 || { cat $OUT/kb32k.log; exit 1; }
grep -E "x2|v9" $OUT/kb32k.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --size 8192 --steps 1000 --skip-extras > $OUT/bench8k.json 2>> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench8k.json
