#!/bin/bash
# Round 5 (s): bisect the 2-rank band-first timeout of bench.py --overlap on:
# the correctness gate's shape in the app (this tree vs build/var/old), then
# bench.py with the session-start kernel library (GMT_LIB), then without the gate.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_s
mkdir -p $OUT
M=/opt/conda/bin/mpirun
B=$R/build/bin/mpi_jacobi2d
: > $OUT/app.log
for v in old new; do
  lp=""; [ $v = old ] && lp=$R/build/var/old
  echo "== gate shape $v" >> $OUT/app.log
  LD_LIBRARY_PATH=$lp timeout -k 10 60 $M -np 2 $B 0 43 --ny=313 --nx=850 --dims=2x1 --tblock --tsteps=20 --transport=ipc --warmup=0 --check >> $OUT/app.log 2>&1
  rc=$?; echo "gate shape $v rc $rc"; [ $rc -ge 124 ] && exit 1
done
grep -E "^==|TIME|timed out|diff|check" $OUT/app.log | head -20
bn() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29631 bench.py --gpus 2 --size 8192 --steps 20 --warmup 5 --skip-extras --overlap on $BX > $OUT/bench_$name.out 2> $OUT/bench_$name.err
  local rc=$?; echo "bench $name rc $rc: $(tail -1 $OUT/bench_$name.out | cut -c1-200)"
  [ $rc -ge 124 ] && exit 1
  return 0
}
BX="" bn old GMT_LIB=$R/build/var/old/libgmt.so
BX="--skip-check" bn new_nogate GMT_NONE=1
echo R05S_OK
