#!/bin/bash
# Round 4 (v): does the headline (20 timed sweeps of 32768^2) depend on how
# warm the GPU is?  --warmup 5 (the driver's) vs 100 vs 400, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_v}
mkdir -p $OUT
for rep in 1 2; do
  for w in 5 100 400; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup $w --skip-extras > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "import json; r=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('rep $rep warmup $w', r['value'], r['ms_per_step'], r['config']['pass_cost_ms'])" | tee -a $OUT/summary.txt
  done
done
