#!/bin/bash
# Round 6 (y): the N = 8 driver shape on one GPU (8 ranks sharing it, the
# 32768^2 domain split 2 x 4 / 4 x 2: interior-x shares run the shared
# hand-off groups, the others one strip per workgroup) — a functional check
# of the round-6 launch shapes through bench.py, timed fields checked.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_y
mkdir -p $OUT
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29631 bench.py --gpus 8 --steps 20 --warmup 5 --skip-extras > $OUT/n8.out 2> $OUT/n8.err || { tail -30 $OUT/n8.err; exit 1; }
tail -1 $OUT/n8.out > $OUT/n8.json
python3 -c "import json; d=json.load(open('$OUT/n8.json')); print(d['value'], d['config'].get('transport'), d['config'].get('parallelism'), d.get('timed_check_mismatches'), d.get('timed_check_max_diff'), d['config'].get('tb_launch'))"
echo R06Y_OK
