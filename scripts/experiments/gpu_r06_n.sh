#!/bin/bash
# Round 6 (n): shared hand-off groups by default (stage-major waves, the
# SH policy of sh_launch) — the whole GPU suite, then same-box A/B against
# the per-strip launch (GMT_TB_SHARED=0), alternating; the planner's
# one-column rule cost on the one-round Dirichlet shapes (SH forced); the
# driver-config bench with and without SH, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_n
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
    for mask in 0 15; do
      for v in base sh; do
        case $v in
          base) envs="GMT_TB_SHARED=0";;
          sh) envs="GMT_TB_SHARED=1";;
        esac
        echo "== $v m$mask $shp" >> $OUT/rates.log
        env $envs timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
  for shp in "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60"; do
    for c in 1.0 1.3 1.6; do
      echo "== c$c m0 $shp" >> $OUT/rates.log
      GMT_TB_SHARED=1 GMT_TB_RULE_COL_COST=$c timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
for v in def 0 def 0; do
  if [ $v = def ]; then envs="GMT_NOTHING=1"; else envs="GMT_TB_SHARED=0"; fi
  env $envs timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$v.out 2> $OUT/bench_$v.err || { tail -30 $OUT/bench_$v.err; exit 1; }
  tail -1 $OUT/bench_$v.out >> $OUT/bench_$v.jsonl
  tail -1 $OUT/bench_$v.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d.get('timed_pass_sclk_mhz'), d.get('timed_check_mismatches'), d.get('stencil_8192_MLUPS'), d.get('stencil_8192_sclk_mhz'), d.get('stencil_8192_check_mismatches'), d['config'].get('pass_plan'))"
done
echo R06N_OK
