#!/bin/bash
# Round 5 (i): the segment planner's rule-path cost after the exec-masked keep
# (GMT_TB_RULE_COST: 1.8 = round 4's select, 1.3 the new default), Dirichlet
# sides against halo sides, alternating, same box; then bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_i
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
    echo "== m15 $shp" >> $OUT/rates.log
    timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=15 $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
    for c in 1.8 1.5 1.3 1.2; do
      echo "== c$c $shp" >> $OUT/rates.log
      GMT_TB_RULE_COST=$c timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out > $OUT/bench.json; cat $OUT/bench.json
