#!/bin/bash
# Round 4 (j): column-band-aware segment planner (band-first passes price a
# plan at max(makespan, 1.25 x the column bands' end) and may shorten the
# band groups' segments) vs HEAD's planner (build/ab_head): bitwise tests,
# then overlap vs serial on the strong-scaling shares, 3 alternating reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_j}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_jacobi_tb_gpu.py tests/test_native_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A40 FAILURES $OUT/pytest.log | head -80; exit $rc; }
: > $OUT/shares.txt
for rep in 1 2 3; do
  for cfg in "8192 16384" "16384 8192" "16384 16384"; do
    set -- $cfg
    for v in head new; do
      lp=""; [ "$v" != new ] && lp=$R/build/ab_$v
      for mode in "--no-overlap" "--overlap"; do
        LD_LIBRARY_PATH=$lp timeout -k 10 200 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 --graph \
          --periodic --transport=rccl $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
        echo "rep=$rep $v ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log)" | tee -a $OUT/shares.txt
      done
    done
  done
done
