#!/bin/bash
# one strip per two-stage workgroup: bitwise tests (kernel + engine band-first),
# the driver bench, and a kernel trace of the N = 8 share inside mpi_jacobi2d
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tb4g}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_jacobi_tb_gpu.py tests/test_native_gpu.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench_driver.json
R=$PWD
M=/opt/conda/bin/mpirun
cd /tmp
for mode in "" "--periodic --transport=rccl --no-overlap"; do
  timeout -k 10 200 $M -np 1 $R/build/bin/mpi_jacobi2d --ny=8192 --nx=16384 100 --tblock --tsteps=20 --warmup=20 --graph $mode > $R/$OUT/j.log 2>&1 || { cat $R/$OUT/j.log; exit 1; }
  echo "share8 [$mode] $(grep -E 'TIME step' $R/$OUT/j.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/prof -o s8 -- $R/build/bin/mpi_jacobi2d --ny=8192 --nx=16384 100 --tblock --tsteps=20 --warmup=20 --graph > $R/$OUT/prof.log 2>&1 || { tail -20 $R/$OUT/prof.log; exit 1; }
echo PROF_OK
