#!/bin/bash
# Round 5 (z): the final tree — TB / push numerics under the planner's
# edges-last plans, rates on the headline domain (planner vs forced off),
# the full GPU suite, smoke and the driver-config bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_z
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for el in "" 0; do
    echo "== el'$el'" >> $OUT/rates.log
    env ${el:+GMT_TB_EDGES_LAST=$el} timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 --jacobi-n=32768 --iters=20 >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out > $OUT/bench.json; cut -c1-600 $OUT/bench.json
