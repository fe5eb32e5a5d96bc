#!/bin/bash
# planner choice vs fixed segment lengths on the strong-scaling shares (K=20),
# 100 back-to-back launches per point, each config measured twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/sharek3
B=build/bin/gmt_kernel_bench
run() {  # tag, args
  local t=$1; shift
  timeout -k 10 200 $B --only=tb --iters=${ITERS:-100} --sustained=1 "$@" > gpurun_out/sharek3/$t.log 2>&1 || { cat gpurun_out/sharek3/$t.log; exit 1; }
  grep MLUPS gpurun_out/sharek3/$t.log | cut -c15-
}
for rep in 1 2; do
run s8_$rep --tb-k=20 --tb-nw=2 --tb-mask=15 --jacobi-ny=8192 --jacobi-nx=16384 --tb-seg=0,512,640,768,1024
run s8t_$rep --tb-k=20 --tb-nw=2 --tb-mask=15 --jacobi-ny=16384 --jacobi-nx=8192 --tb-seg=0,512,768,1024
run s4_$rep --tb-k=20 --tb-nw=2 --tb-mask=15 --jacobi-n=16384 --tb-seg=0,768,1024
run s2_$rep --tb-k=20 --tb-nw=2 --tb-mask=15 --jacobi-ny=16384 --jacobi-nx=32768 --tb-seg=0,768,1024
ITERS=30 run n32_$rep --tb-k=20 --tb-nw=2 --tb-mask=0 --jacobi-n=32768 --tb-seg=0
done
