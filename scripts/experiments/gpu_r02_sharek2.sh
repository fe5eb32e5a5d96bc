#!/bin/bash
# planner choice vs fixed segment lengths on the strong-scaling shares (K=20)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/sharek2
B=build/bin/gmt_kernel_bench
run() {  # tag, args
  local t=$1; shift
  timeout -k 10 200 $B --only=tb --iters=10 --sustained=1 "$@" > gpurun_out/sharek2/$t.log 2>&1 || { cat gpurun_out/sharek2/$t.log; exit 1; }
  grep MLUPS gpurun_out/sharek2/$t.log
}
run n32 --tb-k=20 --tb-nw=0,1,2 --tb-mask=0 --jacobi-n=32768 --tb-seg=0,1024,2048
run s8 --tb-k=20 --tb-nw=1,2,4 --tb-mask=15 --jacobi-ny=8192 --jacobi-nx=16384 --tb-seg=0,384,512,640,768,896,1024,1152,1280,1408,1536
run s8d --tb-k=20 --tb-nw=2 --tb-mask=0 --jacobi-ny=8192 --jacobi-nx=16384 --tb-seg=0,512,768,1024
run n8 --tb-k=20 --tb-nw=1,2 --tb-mask=0 --jacobi-n=8192 --tb-seg=0,256,384,512,768
run s4 --tb-k=20 --tb-nw=2 --tb-mask=15 --jacobi-n=16384 --tb-seg=0,768,1024
