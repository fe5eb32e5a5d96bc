#!/bin/bash
# Round 6 (a): the check of the timed run on the GPU — the production-geometry
# bitwise tests, the push cases through bench.py at 2 ranks sharing the GPU,
# the driver-config bench (timed_check_*), and an injected corrupt ghost cell
# at 32768^2 that must exit 6.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_production_geometry_gpu.py tests/test_multirank_gpu.py -k "production or compare or push" -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.out 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.out > $OUT/bench.json; cut -c1-300 $OUT/bench.json
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
print({k: v for k, v in d.items() if 'check' in k or k.startswith('stencil_')})"
rc=0
GMT_CORRUPT_PASS=0:2 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --skip-check --skip-extras > $OUT/bench_corrupt.out 2> $OUT/bench_corrupt.err || rc=$?
echo "corrupt run rc=$rc"
[ $rc -eq 6 ] || { tail -30 $OUT/bench_corrupt.err; exit 1; }
tail -1 $OUT/bench_corrupt.out | cut -c1-200
grep -o '"timed_check[a-z_]*": [^,]*' $OUT/bench_corrupt.out
echo R06A_OK
