#!/bin/bash
# Round 4 (z): IPC exchange with halo faces moved in place (the exchange
# kernel gathers/scatters strided faces, no pack/unpack launches) vs packed
# (GMT_IPC_BLOCKS=0): GPU tests, then 2 and 4 ranks sharing the GPU,
# periodic 2-D grids, serial order, alternating, 3 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_z}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_native_gpu.py tests/test_multirank_gpu.py tests/test_kernels_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A40 FAILURES $OUT/pytest.log | head -80; exit $rc; }
MPI=/opt/conda/bin/mpirun
: > $OUT/summary.txt
for rep in 1 2 3; do
  for np in 2 4; do
    for b in 1 0; do
      GMT_IPC_BLOCKS=$b timeout -k 10 200 $MPI -np $np build/bin/mpi_jacobi2d --ny=16384 --nx=16384 100 --tblock --tsteps=20 \
        --warmup=20 --periodic --transport=ipc --no-overlap --check > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
      echo "rep=$rep np=$np GMT_IPC_BLOCKS=$b $(grep -E 'TIME step' $OUT/j.log) | $(grep -E '^halo' $OUT/j.log) | $(grep -iE 'max.*diff|check' $OUT/j.log | head -1)" | tee -a $OUT/summary.txt
    done
  done
done
