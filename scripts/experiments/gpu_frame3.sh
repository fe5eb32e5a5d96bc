#!/bin/bash
# shifted strips with the main core's segment length: numerics, timings
# (overlap / no-overlap / graph), bench with and without graphs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/frame3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -m gpu -x -q -k "jacobi5xk or engine or app_jacobi" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
M=/opt/conda/bin/mpirun
for cfg in "32768 32768" "16384 32768" "8192 32768" "8192 16384"; do
  set -- $cfg
  for mode in "" "--graph" "--periodic --transport=rccl" "--periodic --transport=rccl --no-overlap" "--periodic --transport=rccl --graph"; do
    timeout -k 10 200 $M -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 60 --tblock --tsteps=12 --warmup=12 $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log)"
  done
done
timeout -k 10 300 python bench.py --skip-extras > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --skip-extras --graph off > $OUT/bench_eager.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench_eager.json
R=$PWD
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/p -o per -- $R/build/bin/mpi_jacobi2d --ny=8192 --nx=16384 48 --tblock --tsteps=12 --warmup=12 --periodic --transport=rccl > $R/$OUT/per.log 2>&1 || { tail -30 $R/$OUT/per.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/b -o bench -- python3 $R/bench.py --skip-extras --steps 48 > $R/$OUT/bprof.log 2>&1 || { tail -30 $R/$OUT/bprof.log; exit 1; }
echo PROF_OK
