#!/bin/bash
# Round 5 (v): smoke, the driver-config bench (twice), the 2-rank probe
# (gpu_r05_p.sh) and the random/analytic field A/B; kernel stats of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_v
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$rep.out 2> $OUT/bench_$rep.err || { tail -30 $OUT/bench_$rep.err; exit 1; }
  tail -1 $OUT/bench_$rep.out > $OUT/bench_$rep.json; cut -c1-400 $OUT/bench_$rep.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --skip-extras > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
timeout -k 10 300 python -u scripts/experiments/init_ab.py 8192 1000 > $OUT/init_ab_8192.log 2>&1 || { tail -20 $OUT/init_ab_8192.log; exit 1; }
cat $OUT/init_ab_8192.log
timeout -k 10 300 python -u scripts/experiments/init_ab.py 32768 60 > $OUT/init_ab_32768.log 2>&1 || { tail -20 $OUT/init_ab_32768.log; exit 1; }
cat $OUT/init_ab_32768.log
bash scripts/experiments/gpu_r05_p.sh
