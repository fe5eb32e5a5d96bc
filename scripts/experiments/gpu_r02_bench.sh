#!/bin/bash
# bench.py: driver config (20 steps), default (100 steps), tsteps 24, 40 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${1:-gpurun_out/bench}
mkdir -p $OUT
for a in "--gpus 1 --steps 20 --warmup 5" "" "--tsteps 24" "--steps 40 --warmup 5"; do
  timeout -k 10 300 python bench.py $a > $OUT/b.json 2>> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
  n=$(grep -c . $OUT/b.json); [ "$n" = 1 ] || echo "stdout has $n lines"; python -c "import json;d=json.load(open('$OUT/b.json'));print('$a', d['value'], d['config']['pass_plan'], d['stencil_8192_MLUPS'], d['stencil_8192_pass_plan'], d['halo_exchange_us'], d['daxpy_GBps'])"
done
