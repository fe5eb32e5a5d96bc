#!/bin/bash
# Round 5 (u): after the even segment split — the 2-rank bench with band-first
# that hung, the full GPU suite, smoke, the driver-config bench, the 2-rank
# probe runs and the random/analytic A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_u
mkdir -p $OUT
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29641 bench.py --gpus 2 --size 8192 --steps 20 --warmup 5 --daxpy-n 16777216 --ref-iters 20 \
  --overlap on > $OUT/bench_n2_overlap.out 2> $OUT/bench_n2_overlap.err || { tail -5 $OUT/bench_n2_overlap.out; tail -20 $OUT/bench_n2_overlap.err; exit 1; }
tail -1 $OUT/bench_n2_overlap.out | cut -c1-300
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
