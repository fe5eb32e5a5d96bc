#!/bin/bash
# Round 6 (w): the default-shape test and the bench line's launch record.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_w
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_tb_shared_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out > $OUT/bench.json
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['config'].get('tb_launch'), d.get('stencil_8192_MLUPS'), d.get('timed_check_mismatches'))"

bash scripts/experiments/gpu_r06_g.sh
