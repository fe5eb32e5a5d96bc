#!/bin/bash
# Round-1 GPU pass 3: all GPU tests, kernel A/B, smoke, bench.py (native engine), rocprof.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r1b
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 build/bin/gmt_kernel_bench --iters=20 --json=$OUT/kb.jsonl > $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
cat $OUT/kb.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --engine torch --skip-extras > $OUT/bench_torch.json 2>> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench_torch.json
timeout -k 10 300 python bench.py --size 8192 --steps 500 --skip-extras > $OUT/bench_8192.json 2>> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench_8192.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
echo PROF_OK
