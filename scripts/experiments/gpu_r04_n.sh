#!/bin/bash
# Round 4 (n): bench.py's start-up data-plane probe on the GPU (2 and 4
# ranks sharing the box's one MI355X, probe forced on: the IPC candidate in
# an isolated child process group), then the 1-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_n}
mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 --transport-probe on \
    > $OUT/bench_n$n.json 2> $OUT/bench_n$n.err || { tail -30 $OUT/bench_n$n.err; exit 1; }
  python3 -c "import json,sys; r=json.loads([l for l in open('$OUT/bench_n$n.json') if l.startswith('{')][0]); print($n, r['value'], r['config']['transport'], r.get('transport_candidates'), r.get('transport_probe_s'), r['check_max_diff'])"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench1.json 2> $OUT/bench1.err || { tail -20 $OUT/bench1.err; exit 1; }
cat $OUT/bench1.json
