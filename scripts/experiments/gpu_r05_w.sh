#!/bin/bash
# Round 5 (w): the headline domain's Dirichlet plan — balanced edges (the
# model's choice) vs short edges at the halo-side segment length, with and
# without the edge tiles round-robin over the XCDs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_w
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for cfg in "default:" "short1640:GMT_TB_PLAN_L=1640" "short1640_rr:GMT_TB_PLAN_L=1640 GMT_TB_SPECIAL_RR=1" \
             "default_rr:GMT_TB_SPECIAL_RR=1" "short_model:GMT_TB_EDGES=1" "short1600:GMT_TB_PLAN_L=1600" "m15:"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    m=0; [ $name = m15 ] && m=15
    echo "== $name" >> $OUT/rates.log
    env $envs timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$m --jacobi-n=32768 --iters=20 >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2), $(NF-1)}'
