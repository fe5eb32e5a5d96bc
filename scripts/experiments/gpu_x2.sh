#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/x2
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "jacobi5x2 or stencil5" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 build/bin/gmt_kernel_bench --iters=20 --only=jacobi,stencil > $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
cat $OUT/kb.log
timeout -k 10 300 build/bin/gmt_kernel_bench --iters=20 --only=jacobi --jacobi-n=8192 > $OUT/kb8k.log 2>&1 || { cat $OUT/kb8k.log; exit 1; }
cat $OUT/kb8k.log
M=/opt/conda/bin/mpirun
for a in "515 30 --check" "515 31 --check --periodic --graph" "515 30 --check --periodic --graph --transport=rccl" "1000 20 --check --tblock=8"; do
  timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d $a --tblock --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
  grep -E "check|transport" $OUT/jc.log
done
timeout -k 10 120 $M -np 2 build/bin/mpi_jacobi2d 515 30 --check --tblock --transport=ipc --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
grep -E "check|transport" $OUT/jc.log
timeout -k 10 120 $M -np 4 build/bin/mpi_jacobi2d 515 30 --check --tblock --dims=2x2 --periodic --transport=ipc --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
grep -E "check|transport|grid" $OUT/jc.log
for tb in 8 16 32; do
  timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d 32768 100 --tblock=$tb --graph > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
  grep -E "MLUPS|TIME" $OUT/j.log
done
timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d 32768 100 --tblock --periodic --graph --transport=rccl --halo-iters=20 > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
grep -E "MLUPS|TIME|halo" $OUT/j.log
timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d 8192 400 --tblock --graph > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
grep -E "MLUPS|TIME" $OUT/j.log
