#!/bin/bash
# Round 6 (c): the segment planner's rule-path cost above round 5's sweep
# (which rose monotonically to its top value 1.8 at 8192^2), Dirichlet sides,
# alternating reps, same box; the kernel trace of the 8192^2 bench pattern
# (1000 sweeps = 50 passes: kernel time against wall time).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_c
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60" "--jacobi-n=32768 --iters=20"; do
    for c in 1.8 2.1 2.4 2.8 3.3; do
      echo "== c$c $shp" >> $OUT/rates.log
      GMT_TB_RULE_COST=$c timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
cd $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace8192 -o t -- python3 $R/scripts/experiments/clock_ab.py 8192 1000 2 > $OUT/trace8192.log 2>&1 || { tail -20 $OUT/trace8192.log; exit 1; }
grep "^n " $OUT/trace8192.log
echo R06C_OK
