#!/bin/bash
# Round 5 (p): bench.py at 2 ranks sharing the GPU, three runs: which data
# plane does the start-up probe pick (--transport-probe on; rccl is out: two ranks on one GPU),
# ipc (serial exchange kernel) or push (inline halo)?
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r05_p}
mkdir -p $OUT
for rep in 1 2 3; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + rep)) bench.py --gpus 2 --steps 20 --warmup 5 --skip-extras --transport-probe on > $OUT/bench_n2_$rep.out 2> $OUT/bench_n2_$rep.err || { tail -30 $OUT/bench_n2_$rep.err; exit 1; }
  tail -1 $OUT/bench_n2_$rep.out > $OUT/bench_n2_$rep.json
  python3 -c "
import json; d = json.load(open('$OUT/bench_n2_$rep.json'))
print('rep $rep', d['value'], d['config'].get('transport'), json.dumps(d.get('transport_candidates')))"
done
echo R05P_OK
