#!/bin/bash
# Round 5 (aa): the inline halo's planner cost at application level
# (mpi_jacobi2d one rank periodic, 2000 steps): GMT_TB_PUSH_COST 1.1 / 1.15 /
# 1.2 / 1.3 against the serial RCCL order, alternating, two shares.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_aa
mkdir -p $OUT
M=/opt/conda/bin/mpirun
B=$R/build/bin/mpi_jacobi2d
: > $OUT/app.log
for rep in 1 2; do
  for shp in "--ny=8192 --nx=16384" "--ny=16384 --nx=8192"; do
    for mode in "serial:--no-overlap:1.15" "p1.10:--push:1.10" "p1.15:--push:1.15" "p1.20:--push:1.20" "p1.30:--push:1.30"; do
      name=${mode%%:*}; rest=${mode#*:}; opts=${rest%%:*}; c=${rest#*:}
      echo "== $name $shp" >> $OUT/app.log
      GMT_TB_PUSH_COST=$c timeout -k 10 120 $M -np 1 $B 0 2000 $shp --periodic --tblock --tsteps=20 --warmup=100 \
        --transport=rccl $opts >> $OUT/app.log 2>&1 || { tail -20 $OUT/app.log; exit 1; }
    done
  done
done
grep -E "^==|TIME step" $OUT/app.log | paste - - | awk '{print $2, $3, $4, $(NF-1)}'
