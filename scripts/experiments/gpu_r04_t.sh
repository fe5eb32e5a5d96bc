#!/bin/bash
# Round 4 (t): bench.py's 8192^2 extra timed over 100 steps (default: 1.4 ms
# of GPU work) vs 1000 and 2000 steps, alternating, 2 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_t}
mkdir -p $OUT
for rep in 1 2; do
  for n in 100 1000 2000; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --skip-check --small-steps $n > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "import json; r=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('rep $rep small-steps $n', r['value'], r['stencil_8192_MLUPS'], r['stencil_8192_pass_plan'])" | tee -a $OUT/summary.txt
  done
done
