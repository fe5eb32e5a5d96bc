#!/bin/bash
# Round 5 (cc): the derivative stencils' box-to-box spread — five reps of the
# reference-shape dim-0 / dim-1 kernels with DAXPY as the HBM yardstick on the
# same box, then bytes moved per kernel (FETCH_SIZE, WRITE_SIZE in passes of
# their own).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_cc
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2 3 4 5; do
  timeout -k 10 120 $B --only=stencil,daxpy --iters=50 >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
done
grep -E "stencil5|daxpy" $OUT/rates.log | head -30
cd $OUT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o fetch --output-format csv -- $B --only=stencil --iters=5 > $OUT/pmc_fetch.log 2>&1 || { tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o write --output-format csv -- $B --only=stencil --iters=5 > $OUT/pmc_write.log 2>&1 || { tail -20 $OUT/pmc_write.log; exit 1; }
echo R05CC_OK
