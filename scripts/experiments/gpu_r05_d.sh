#!/bin/bash
# Round 5 (d): the planner's balanced edge segments against short ones
# (build/var/short: the same library with the long-edge search off; build/var/head:
# the committed kernel, per-cell rule select), same
# box, alternating; then the driver-config bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r05_d}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for v in ${VARIANTS:-new head short}; do
    lp=""; [ "$v" != new ] && lp=$R/build/var/$v
    for m in 0 15; do
      for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
        echo "== $v m$m $shp" >> $OUT/rates.log
        LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$m $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-12), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out > $OUT/bench.json; cat $OUT/bench.json
