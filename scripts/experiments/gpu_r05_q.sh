#!/bin/bash
# Round 5 (q): the failing oversubscribed bench (2 ranks, --overlap on),
# full output kept; then the 2-rank probe runs (gpu_r05_p.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r05_q
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_native_gpu.py -k "band or overlap" \
  > $OUT/pytest_band.log 2>&1
rc=$?; echo "band tests exit $rc"; tail -3 $OUT/pytest_band.log; grep -E "^FAILED" $OUT/pytest_band.log | head
[ $rc -ge 2 ] && exit 1  # a time limit, a crash or an internal error: no further GPU step
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --size 8192 --steps 20 --warmup 5 --daxpy-n 16777216 --ref-iters 20 \
  --overlap on > $OUT/n2_overlap.out 2> $OUT/n2_overlap.err
rc=$?; echo "exit $rc"
tail -3 $OUT/n2_overlap.out | cut -c1-3000
grep -n "probe\|transport\|failed\|timed out" $OUT/n2_overlap.out $OUT/n2_overlap.err | head -20
[ $rc -ge 124 ] && exit 1
bash scripts/experiments/gpu_r05_p.sh
