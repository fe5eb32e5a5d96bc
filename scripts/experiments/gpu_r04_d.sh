#!/bin/bash
# Round 4 (d: hand-off writes left in flight across the barrier, lag 3): the wide K = 20 kernel (6 columns per lane, 4 stages, sliding
# input rows).  Bitwise tests of every K, engine --check runs at K = 20,
# then sustained K = 20 rates against the round-3 kernel (build/ab_r03, and the two-strip workgroup shape new2,
# scripts/build_variant.sh r03 git:<round-3 head>), alternating twice, then
# the driver's bench config.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/r04_d}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jacobi_tb_gpu.py > $OUT/pytest_tb.log 2>&1 || { tail -30 $OUT/pytest_tb.log; exit 1; }
tail -2 $OUT/pytest_tb.log
chk() {  # run mpi_jacobi2d --check, require max|diff| == 0
  timeout -k 10 120 "$@" > $OUT/chk.log 2>&1 || { cat $OUT/chk.log; echo "FAILED: $*"; exit 1; }
  d=$(grep -oE "vs serial = [0-9.e+-]+" $OUT/chk.log | awk '{print $4}')
  echo "$d  $*" | tee -a $OUT/checks.txt
  python3 -c "import sys; sys.exit(0 if float('$d') == 0.0 else 1)" || { cat $OUT/chk.log; echo "NOT BITWISE: $*"; exit 1; }
}
: > $OUT/checks.txt
chk build/bin/mpi_jacobi2d --ny=700 --nx=1900 0 47 --check --tblock --tsteps=20
chk build/bin/mpi_jacobi2d --ny=700 --nx=1900 0 47 --check --tblock --tsteps=20 --periodic
chk build/bin/mpi_jacobi2d --ny=333 --nx=517 0 41 --check --tblock --tsteps=20
chk build/bin/mpi_jacobi2d --ny=1500 --nx=1900 0 47 --check --tblock --tsteps=20 --periodic --transport=rccl --overlap
chk build/bin/mpi_jacobi2d --ny=1500 --nx=1900 0 47 --check --tblock --tsteps=20 --periodic=x --transport=rccl --overlap
chk $M -np 2 build/bin/mpi_jacobi2d --ny=701 --nx=1900 0 47 --check --tblock --tsteps=20 --transport=ipc --dims=2x1
chk $M -np 2 build/bin/mpi_jacobi2d --ny=701 --nx=1900 0 47 --check --tblock --tsteps=20 --transport=ipc --dims=1x2
B=build/bin/gmt_kernel_bench
for rep in 1 2; do
  for v in r03 new new2; do
    lp=""; NW=0; [ "$v" = r03 ] && lp=build/ab_r03; [ "$v" = new2 ] && NW=2
    : > $OUT/$v.$rep.log
    for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=100" "--jacobi-n=8192 --iters=100"; do
      LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 --tb-nw=$NW $shp >> $OUT/$v.$rep.log 2>&1 || { cat $OUT/$v.$rep.log; exit 1; }
    done
    echo "$v: $(grep MLUPS $OUT/$v.$rep.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
  done
done
grep MLUPS $OUT/new.1.log $OUT/new2.1.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_native_gpu.py -k "halo_check" > $OUT/pytest_check.log 2>&1 || { tail -30 $OUT/pytest_check.log; exit 1; }
tail -2 $OUT/pytest_check.log
