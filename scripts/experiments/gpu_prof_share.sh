#!/bin/bash
# rocprofv3 kernel trace of the N=8 per-GPU share (8192 x 16384, periodic
# self-exchange over RCCL, eager, K=12) and of the Dirichlet single-rank run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$PWD
OUT=$R/gpurun_out/profshare
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o per -- $R/build/bin/mpi_jacobi2d --ny=8192 --nx=16384 48 --tblock --tsteps=12 --warmup=12 --periodic --transport=rccl > $OUT/per.log 2>&1 || { tail -30 $OUT/per.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/d -o dir -- $R/build/bin/mpi_jacobi2d --ny=8192 --nx=16384 48 --tblock --tsteps=12 --warmup=12 > $OUT/dir.log 2>&1 || { tail -30 $OUT/dir.log; exit 1; }
grep -E "TIME step" $OUT/per.log $OUT/dir.log
find $OUT -name "*.csv" | head
