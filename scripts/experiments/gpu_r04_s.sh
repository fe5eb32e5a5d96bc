#!/bin/bash
# Round 4 (s): bench.py's 8192^2 rate with the calibrated pass plan vs the
# built-in cost table (--no-calibrate), alternating, 2 reps each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_s}
mkdir -p $OUT
for rep in 1 2; do
  for c in "" "--no-calibrate"; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-check $c > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "import json; r=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('rep $rep [$c]', r['value'], r['config']['pass_plan'], r['config']['pass_cost_ms'], r['stencil_8192_MLUPS'], r['stencil_8192_pass_plan'])" | tee -a $OUT/summary.txt
  done
done
