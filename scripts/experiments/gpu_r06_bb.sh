#!/bin/bash
# Round 6 (bb): the N = 2 and N = 4 driver shapes on one GPU through
# bench.py with the final launch defaults (ranks sharing the GPU; timed
# fields checked) — functional, not scaling.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_bb
mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29640 + n)) bench.py --gpus $n --steps 20 --warmup 5 --skip-extras > $OUT/n$n.out 2> $OUT/n$n.err || { tail -30 $OUT/n$n.err; exit 1; }
  tail -1 $OUT/n$n.out > $OUT/n$n.json
  python3 -c "import json; d=json.load(open('$OUT/n$n.json')); print($n, d['value'], d['config'].get('transport'), d['config'].get('parallelism'), d.get('timed_check_mismatches'), d['config'].get('tb_launch', {}).get('threads'), d.get('timed_pass_sclk_mhz'))"
done
echo R06BB_OK
