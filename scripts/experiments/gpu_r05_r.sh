#!/bin/bash
# Round 5 (r): band-first at 2 ranks sharing the GPU (bench.py --overlap on
# timed out waiting for its boundary bands): the app on the same shares,
# this tree's K = 20 kernel vs the session-start one (build/var/old), and
# with the planner's rule cost / length pinned.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_r
mkdir -p $OUT
M=/opt/conda/bin/mpirun
B=$R/build/bin/mpi_jacobi2d
run() {  # name, env..., then args
  local name=$1; shift
  echo "== $name" >> $OUT/app.log
  timeout -k 10 90 env "$@" >> $OUT/app.log 2>&1
  local rc=$?
  echo "rc $rc" >> $OUT/app.log
  grep -E "TIME step|timed out|error" $OUT/app.log | tail -2
  [ $rc -ge 124 ] && exit 1
  return 0
}
: > $OUT/app.log
A="--ny=8192 --nx=8192 --dims=2x1 --tblock --tsteps=20 --transport=ipc --warmup=40"
for rep in 1 2; do
  run old LD_LIBRARY_PATH=$R/build/var/old $M -np 2 $B 0 400 $A
  run new $M -np 2 $B 0 400 $A
done
run new_serial $M -np 2 $B 0 400 $A --no-overlap
for rep in 1 2; do
  echo "== bench n2 overlap on, rep $rep" >> $OUT/app.log
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29620 + rep)) bench.py --gpus 2 --size 8192 --steps 20 --warmup 5 --daxpy-n 16777216 --ref-iters 20 \
    --overlap on > $OUT/bench_$rep.out 2> $OUT/bench_$rep.err
  rc=$?; echo "bench rep $rep rc $rc"; tail -2 $OUT/bench_$rep.out | cut -c1-300
  [ $rc -ge 124 ] && exit 1
done
echo R05R_OK
