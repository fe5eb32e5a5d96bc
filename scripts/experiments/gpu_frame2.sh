#!/bin/bash
# one-phase corner exchange + core-after-pack ordering: numerics, A/B timings
# of the per-GPU share, kernel traces, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/frame2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -m gpu -x -q -k "jacobi5xk or engine or app_jacobi" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
M=/opt/conda/bin/mpirun
for cfg in "32768 32768" "16384 32768" "8192 32768" "8192 16384"; do
  set -- $cfg
  for mode in "" "--periodic --transport=rccl" "--periodic --transport=rccl --no-overlap" "--periodic --transport=rccl --graph"; do
    for envs in "X=1" "GMT_CORE_AFTER_PACK=0" "GMT_HALO_TWO_PHASE=1"; do
      [ -z "$mode" ] && [ "$envs" != "X=1" ] && continue
      timeout -k 10 200 env $envs $M -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 60 --tblock --tsteps=12 --warmup=12 $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
      echo "ny=$1 nx=$2 [$mode] $envs $(grep -E 'TIME step' $OUT/j.log)"
    done
  done
done
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
R=$PWD
cd /tmp
for v in 1 0; do
GMT_CORE_AFTER_PACK=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/p$v -o per -- $R/build/bin/mpi_jacobi2d --ny=8192 --nx=16384 48 --tblock --tsteps=12 --warmup=12 --periodic --transport=rccl > $R/$OUT/per$v.log 2>&1 || { tail -30 $R/$OUT/per$v.log; exit 1; }
done
echo PROF_OK
