#!/bin/bash
# Round 3: is the Jacobi rate data-independent?  Driver config (20 steps) and
# the 100-step default, random-init vs analytic field, alternating A B A B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r03_init_ab
mkdir -p $OUT
for rep in 1 2; do
  for init in random analytic; do
    for steps in 20 100; do
      timeout -k 10 180 python -u bench.py --gpus 1 --steps $steps --warmup 5 --init $init --skip-extras \
        > $OUT/b_${init}_${steps}_$rep.out 2> $OUT/b_${init}_${steps}_$rep.err || { tail -20 $OUT/b_${init}_${steps}_$rep.err; exit 1; }
      python -c "import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], r['value'], r['ms_per_step'], r['config']['pass_plan'], r['check_max_diff'], r['config']['max_abs_u0'])" \
        $OUT/b_${init}_${steps}_$rep.out $rep $init $steps | tee -a $OUT/summary.txt
    done
  done
done
