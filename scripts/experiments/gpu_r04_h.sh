#!/bin/bash
# Round 4 (h): makespan segment planner + rule workgroups dispatched over all
# XCDs (production) vs the round-3 planner (build/ab_base = HEAD before it):
# bitwise tests, sustained K = 20 rates on the four shapes (Dirichlet sides:
# mask 0; all halo sides: mask 15), the strong-scaling shares, the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_h}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_jacobi_tb_gpu.py tests/test_native_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A40 FAILURES $OUT/pytest.log | head -80; exit $rc; }
B=$R/build/bin/gmt_kernel_bench
for rep in 1 2; do
  for v in base new; do
    lp=""; [ "$v" != new ] && lp=$R/build/ab_$v
    for m in 0 15; do
      : > $OUT/$v.m$m.$rep.log
      for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=100" "--jacobi-n=8192 --iters=100"; do
        LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$m $shp >> $OUT/$v.m$m.$rep.log 2>&1 || { cat $OUT/$v.m$m.$rep.log; exit 1; }
      done
      echo "$v mask $m: $(grep MLUPS $OUT/$v.m$m.$rep.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
    done
  done
done
grep MLUPS $OUT/new.m0.1.log $OUT/base.m0.1.log
: > $OUT/shares.txt
for cfg in "32768 32768" "16384 32768" "16384 16384" "8192 16384" "16384 8192"; do
  set -- $cfg
  for mode in "--no-overlap" "--overlap"; do
    timeout -k 10 200 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 --graph \
      --periodic --transport=rccl $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log)" | tee -a $OUT/shares.txt
  done
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
