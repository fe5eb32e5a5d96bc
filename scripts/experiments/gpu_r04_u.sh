#!/bin/bash
# Round 4 (u): the share table again with the kernel bench's first
# measurement warmed up (200 ms of launches): every shape in its own
# process, masks 0 and 15, 2 reps; then the 1-GPU bench (8192^2 extra over
# 1000 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_u}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/shares.txt
for rep in 1 2; do
  for m in 0 15; do
    for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=100" "--jacobi-n=8192 --iters=100"; do
      timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$m $shp > $OUT/s.log 2>&1 || { cat $OUT/s.log; exit 1; }
      grep MLUPS $OUT/s.log | sed "s/^/rep=$rep /" | tee -a $OUT/shares.txt
    done
  done
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
