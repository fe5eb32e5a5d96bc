#!/bin/bash
# Round 6 (g): the data-plane probe at 2 ranks sharing the GPU, three runs
# (--transport-probe on: ipc and push, each twice in the order A B B A): does
# it pick the same plane three times, or report a tie?
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_g
mkdir -p $OUT
for rep in 1 2 3; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29600 + rep)) bench.py --gpus 2 --steps 20 --warmup 5 --skip-extras --transport-probe on > $OUT/probe_n2_$rep.out 2> $OUT/probe_n2_$rep.err || { tail -30 $OUT/probe_n2_$rep.err; exit 1; }
  tail -1 $OUT/probe_n2_$rep.out > $OUT/probe_n2_$rep.json
  python3 -c "
import json; d = json.load(open('$OUT/probe_n2_$rep.json'))
c = d.get('transport_candidates') or {}
print('rep $rep', d['value'], d['config'].get('transport'), d.get('timed_check_mismatches'), d.get('timed_pass_sclk_mhz'),
      {k: (v.get('pass_ms_reps'), v.get('gate')) for k, v in c.items()}, d.get('transport_probe_s'))"
done
echo R06G_OK
