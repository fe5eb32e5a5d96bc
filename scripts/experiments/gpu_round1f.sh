#!/bin/bash
# Round-1 verification final round-1 pass: scaled K=14 pipeline, overlap auto-tune: GPU tests, smoke, bench.py
# (default), native app validation, rocprofv3 kernel stats of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/r1f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash scripts/gpu_native.sh > $OUT/native.out 2>&1 || { tail -30 $OUT/native.out; exit 1; }
tail -1 $OUT/native.out
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
echo PROF_OK
M=/opt/conda/bin/mpirun
cd $GRAFT_REPO_ROOT
for cfg in "16384 32768" "8192 32768" "8192 16384"; do
  set -- $cfg
  timeout -k 10 200 $M -np 1 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=14 --warmup=14 --periodic --transport=rccl --overlap=auto > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
  echo "share ny=$1 nx=$2 auto: $(grep -E 'TIME step|transport' $OUT/j.log | tr '\n' ' ')"
done
