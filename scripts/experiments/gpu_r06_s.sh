#!/bin/bash
# Round 6 (s): push passes with the two-strip default (shares over 2^28
# points) — push kernel tests incl. several strips per workgroup, then
# bench.py at two ranks sharing the GPU with push and with IPC (16384 x
# 32768 shares: the two-strip shape), timed fields checked.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_s
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_push_gpu.py tests/test_production_geometry_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for t in push ipc push ipc; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --skip-extras --transport $t > $OUT/n2_$t.out 2> $OUT/n2_$t.err || { tail -30 $OUT/n2_$t.err; exit 1; }
  tail -1 $OUT/n2_$t.out >> $OUT/n2_$t.jsonl
  tail -1 $OUT/n2_$t.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['config'].get('transport'), d.get('timed_pass_sclk_mhz'), d.get('timed_check_mismatches'), d['config'].get('pass_plan'), d['config'].get('parallelism'))"
done
echo R06S_OK
