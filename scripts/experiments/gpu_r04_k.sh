#!/bin/bash
# Round 4 (k): kernel traces of band-first (overlap) and serial passes on the
# N = 8 share 8192 x 16384 (1-rank periodic RCCL self-exchange): when do the
# exchange's kernels run relative to the pass that should hide them?
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_k}
mkdir -p $OUT
for mode in overlap no-overlap; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$mode -o tr -- \
    build/bin/mpi_jacobi2d --ny=8192 --nx=16384 200 --tblock --tsteps=20 --warmup=20 \
    --periodic --transport=rccl --$mode > $OUT/$mode.log 2>&1 || { tail -20 $OUT/$mode.log; exit 1; }
  grep "TIME step" $OUT/$mode.log
done
find $OUT -name "*kernel_trace.csv" | head
