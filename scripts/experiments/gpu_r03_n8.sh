#!/bin/bash
# Round 3: bench.py in the driver's N = 8 shape (default 4x2 grid, swapped
# 2x4 timed too), 8 ranks sharing cuda:0 over IPC.  Functional rehearsal of
# the 8-GPU run's control flow, not a scaling number.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r03_n8
mkdir -p $OUT
export OMP_NUM_THREADS=1
timeout -k 10 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 8 --size 8192 --steps 20 --warmup 5 --daxpy-n 16777216 --ref-iters 20 \
  > $OUT/n8.out 2> $OUT/n8.err || { tail -40 $OUT/n8.err; exit 1; }
grep '^{' $OUT/n8.out > $OUT/n8.json; cat $OUT/n8.json
