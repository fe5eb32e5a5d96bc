#!/bin/bash
# Round 4 (aa): pass-cost calibration with ~4 ms of work per measurement:
# the 8192^2 extra's plan and rate, and the headline, 3 runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_aa}
mkdir -p $OUT
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "import json; r=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('rep $rep', r['value'], r['config']['pass_plan'], r['stencil_8192_MLUPS'], r['stencil_8192_pass_plan'])" | tee -a $OUT/summary.txt
done
