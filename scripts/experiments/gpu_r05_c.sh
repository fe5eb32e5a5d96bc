#!/bin/bash
# Round 5 (c): the inline halo exchange (gmt_tb_opts.push) on the GPU.
#  1. numerics: push kernels and engine (tests/test_push_gpu.py), the TB
#     kernel's bitwise tests, the resource guard;
#  2. cost on the N = 8 shares (one rank, periodic, 20-sweep passes):
#     serial RCCL self-exchange vs band-first vs inline halo, against the
#     kernel alone with halo sides (no exchange at all);
#  3. two ranks sharing the GPU over IPC: serial vs band-first vs inline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r05_c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_push_gpu.py \
  tests/test_kernel_resources.py > $OUT/pytest_push.log 2>&1 || { tail -50 $OUT/pytest_push.log; exit 1; }
tail -2 $OUT/pytest_push.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_jacobi_tb_gpu.py \
  > $OUT/pytest_tb.log 2>&1 || { tail -40 $OUT/pytest_tb.log; exit 1; }
tail -1 $OUT/pytest_tb.log
B=$R/build/bin
MPIRUN=/opt/conda/bin/mpirun
: > $OUT/shares.log
for rep in 1 2; do
  for shp in "--ny=8192 --nx=16384" "--ny=16384 --nx=8192"; do
    echo "== kernel m15 $shp" >> $OUT/shares.log
    ny=$(echo $shp | sed 's/.*--ny=\([0-9]*\).*/\1/'); nx=$(echo $shp | sed 's/.*--nx=\([0-9]*\).*/\1/')
    timeout -k 10 120 $B/gmt_kernel_bench --only=tb --sustained=1 --tb-k=20 --tb-mask=15 --jacobi-ny=$ny --jacobi-nx=$nx --iters=100 >> $OUT/shares.log 2>&1 || { tail -20 $OUT/shares.log; exit 1; }
    for mode in "serial:--transport=rccl --no-overlap" "band:--transport=rccl" "push:--push --transport=rccl"; do
      name=${mode%%:*}; opts=${mode#*:}
      echo "== $name $shp" >> $OUT/shares.log
      timeout -k 10 120 $MPIRUN -np 1 $B/mpi_jacobi2d 0 200 $shp --periodic --tblock --tsteps=20 --warmup=40 $opts \
        --json=$OUT/shares.json >> $OUT/shares.log 2>&1 || { tail -20 $OUT/shares.log; exit 1; }
    done
  done
done
grep -E "^==|TIME step|MLUPS|x20 nw0" $OUT/shares.log > $OUT/shares_summary.txt
cat $OUT/shares_summary.txt
: > $OUT/two_ranks.log
for rep in 1 2; do
  for mode in "serial:--no-overlap" "band:--overlap" "push:--push"; do
    name=${mode%%:*}; opts=${mode#*:}
    echo "== 2 ranks $name" >> $OUT/two_ranks.log
    timeout -k 10 150 $MPIRUN -np 2 $B/mpi_jacobi2d 0 200 --ny=16384 --nx=16384 --dims=2x1 --periodic --tblock \
      --tsteps=20 --warmup=40 --transport=ipc $opts --json=$OUT/two_ranks.json >> $OUT/two_ranks.log 2>&1 || { tail -20 $OUT/two_ranks.log; exit 1; }
  done
done
grep -E "^==|TIME step|transport" $OUT/two_ranks.log
echo R05C_OK
