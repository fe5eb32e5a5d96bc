#!/bin/bash
# kernel-only K=20 passes on the strong-scaling shares, all-halo (mask 15,
# the periodic share) vs Dirichlet (mask 0): strips per WG x segment length
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/sharek
B=build/bin/gmt_kernel_bench
run() {  # tag, args
  local t=$1; shift
  timeout -k 10 200 $B --only=tb --iters=10 --sustained=1 "$@" > gpurun_out/sharek/$t.log 2>&1 || { cat gpurun_out/sharek/$t.log; exit 1; }
  grep MLUPS gpurun_out/sharek/$t.log
}
run base --tb-k=20 --tb-nw=0 --tb-mask=0 --jacobi-n=32768 --tb-seg=0
run base15 --tb-k=20 --tb-nw=0 --tb-mask=15 --jacobi-n=32768 --tb-seg=0
run s8 --tb-k=16,20,24 --tb-nw=1,2,3,4 --tb-mask=15 --jacobi-ny=8192 --jacobi-nx=16384 --tb-seg=0,256,512,1024,2048,8192
run s8t --tb-k=20 --tb-nw=1,2,4 --tb-mask=15 --jacobi-ny=16384 --jacobi-nx=8192 --tb-seg=0,512,1024,2048
run s4 --tb-k=20 --tb-nw=1,2,4 --tb-mask=15 --jacobi-n=16384 --tb-seg=0,512,1024,2048
