#!/bin/bash
# Round 3: band-first passes with row bands (S/N halo sides signal from the
# main rect's own first/last segments, no band rects): correctness on the GPU,
# then the strong-scaling shares on one GPU (as profiles/r02_shares.md:
# Dirichlet no exchange / periodic RCCL self-exchange serial / band-first / auto).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03_band}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_jacobi_tb_gpu.py "tests/test_native_gpu.py" tests/test_multirank_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A30 FAILURES $OUT/pytest.log | head -60; exit $rc; }
M=/opt/conda/bin/mpirun
K=20
: > $OUT/shares.txt
for cfg in "32768 32768" "16384 32768" "16384 16384" "8192 16384" "16384 8192"; do
  set -- $cfg
  for mode in "" "--periodic --transport=rccl --no-overlap" "--periodic --transport=rccl" "--periodic --transport=rccl --overlap=auto"; do
    timeout -k 10 200 $M -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=$K --warmup=$K --graph $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
    echo "ny=$1 nx=$2 [$mode] $(grep -E 'TIME step|overlap' $OUT/j.log | tr '\n' ' ')" | tee -a $OUT/shares.txt
  done
done
