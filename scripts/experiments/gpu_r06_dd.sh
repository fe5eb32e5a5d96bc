#!/bin/bash
# Round 6 (dd): two-strip shared groups from 2^28 points on — group tests,
# production geometry, the N = 4 driver shape on one GPU, the driver config.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_dd
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_tb_shared_gpu.py tests/test_production_geometry_gpu.py tests/test_jacobi_tb_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29654 bench.py --gpus 4 --steps 20 --warmup 5 --skip-extras > $OUT/n4.out 2> $OUT/n4.err || { tail -30 $OUT/n4.err; exit 1; }
tail -1 $OUT/n4.out > $OUT/n4.json
python3 -c "import json; d=json.load(open('$OUT/n4.json')); print(4, d['value'], d['config'].get('transport'), d['config'].get('parallelism'), d.get('timed_check_mismatches'), d['config'].get('tb_launch', {}).get('threads'))"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out > $OUT/bench.json
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(1, d['value'], d.get('timed_pass_sclk_mhz'), d.get('timed_check_mismatches'), d.get('stencil_8192_MLUPS'), d['config'].get('tb_launch', {}).get('threads'))"
echo R06DD_OK
