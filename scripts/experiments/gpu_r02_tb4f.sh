#!/bin/bash
# 4-column kernel: launch-shape sweep (strips per workgroup, segment rows) on
# the full domain and on the N = 2/4/8 strong-scaling shares, K = 20
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/tb4f}
mkdir -p $OUT
B=build/bin/gmt_kernel_bench
run() {  # tag, args
  local t=$1; shift
  timeout -k 10 200 $B --only=tb --sustained=1 "$@" > $OUT/$t.log 2>&1 || { cat $OUT/$t.log; exit 1; }
  echo "$t: $(grep MLUPS $OUT/$t.log | cut -c15- | tr '\n' '|')"
}
run n32_nw --iters=20 --tb-k=20 --tb-nw=1,2,3,4 --tb-mask=0 --jacobi-n=32768
run n32_h --iters=20 --tb-k=20 --tb-nw=2 --tb-mask=15 --jacobi-n=32768
run n32_seg --iters=20 --tb-k=20 --tb-nw=2 --tb-mask=0 --jacobi-n=32768 --tb-seg=0,256,384,768,1024
run s8 --iters=100 --tb-k=20 --tb-nw=1,2,4 --tb-mask=0 --jacobi-ny=8192 --jacobi-nx=16384
run s8h --iters=100 --tb-k=20 --tb-nw=1,2,4 --tb-mask=15 --jacobi-ny=8192 --jacobi-nx=16384 --tb-seg=0,256,512,1024,2048
run s8m --iters=100 --tb-k=20 --tb-nw=2 --tb-mask=6 --jacobi-ny=8192 --jacobi-nx=16384
run s4 --iters=60 --tb-k=20 --tb-nw=1,2,4 --tb-mask=0 --jacobi-n=16384
run n8k --iters=100 --tb-k=12,14,16,18,20 --tb-nw=1,2 --tb-mask=0 --jacobi-n=8192
