#!/bin/bash
# Round 5 (x): 8192^2 Dirichlet (the BASELINE single-GPU config), one-round
# launch: short vs balanced edge segments, and rule costs 1.5 / 2.2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_x
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2 3; do
  for cfg in "default:" "balanced:GMT_TB_EDGES=2" "short:GMT_TB_EDGES=1" "c2.2:GMT_TB_RULE_COST=2.2" "c2.2bal:GMT_TB_RULE_COST=2.2 GMT_TB_EDGES=2" "m15:"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    m=0; [ $name = m15 ] && m=15
    echo "== $name" >> $OUT/rates.log
    env $envs timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$m --jacobi-n=8192 --iters=200 >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
