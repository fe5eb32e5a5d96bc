#!/bin/bash
# Round 6, final tree (two-strip shared groups by default for large
# Dirichlet passes): the GPU suite, smoke, the driver-config bench three
# times alternating with the previous default (GMT_TB_SHARED=0: two plain
# stage-major strips).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_final3
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for v in def nw2 def nw2 def nw2; do
  if [ $v = def ]; then envs="GMT_NOTHING=1"; else envs="GMT_TB_SHARED=0"; fi
  env $envs timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$v.out 2> $OUT/bench_$v.err || { tail -30 $OUT/bench_$v.err; exit 1; }
  tail -1 $OUT/bench_$v.out >> $OUT/bench_$v.jsonl
  tail -1 $OUT/bench_$v.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d.get('timed_pass_sclk_mhz'), d.get('timed_check_mismatches'), d.get('stencil_8192_MLUPS'), d.get('stencil_8192_check_mismatches'), d['config'].get('tb_launch', {}).get('threads'), d['config'].get('pass_plan'))"
done
echo R06FINAL3_OK
