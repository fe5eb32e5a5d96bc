#!/bin/bash
# Round 6 (q): the launch defaults (two-strip stage-major workgroups for
# large Dirichlet passes, shared hand-off groups for x-halo passes) — the
# whole GPU suite, smoke, then the driver-config bench three times against
# the round-5 launch shape (GMT_TB_STRIP_MAP=0 GMT_TB_SHARED=0), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_q
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for v in def old def old def old; do
  if [ $v = def ]; then envs="GMT_NOTHING=1"; else envs="GMT_TB_SHARED=0 GMT_TB_STRIP_MAP=0"; fi
  env $envs timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$v.out 2> $OUT/bench_$v.err || { tail -30 $OUT/bench_$v.err; exit 1; }
  tail -1 $OUT/bench_$v.out >> $OUT/bench_$v.jsonl
  tail -1 $OUT/bench_$v.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d.get('timed_pass_sclk_mhz'), d.get('timed_check_mismatches'), d.get('stencil_8192_MLUPS'), d.get('stencil_8192_sclk_mhz'), d.get('stencil_8192_check_mismatches'), d['config'].get('pass_plan'), d.get('daxpy_GBps'))"
done
echo R06Q_OK
