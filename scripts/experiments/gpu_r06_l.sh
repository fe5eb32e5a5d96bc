#!/bin/bash
# Round 6 (l): shared hand-off group launches (Sh<K>) — bitwise tests, then
# same-box A/B against the per-strip launch (GMT_TB_SHARED=0), alternating,
# Dirichlet and halo sides, the BASELINE domains and the N = 8 shares; then
# the driver-config bench both ways.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_tb_shared_gpu.py tests/test_jacobi_tb_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60"; do
    for mask in 0 15; do
      for v in 1 0; do
        echo "== sh$v m$mask $shp" >> $OUT/rates.log
        GMT_TB_SHARED=$v timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
for v in 1 0; do
  GMT_TB_SHARED=$v timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_sh$v.out 2> $OUT/bench_sh$v.err || { tail -30 $OUT/bench_sh$v.err; exit 1; }
  tail -1 $OUT/bench_sh$v.out > $OUT/bench_sh$v.json
  python3 -c "import json; d=json.load(open('$OUT/bench_sh$v.json')); print('sh$v', d['value'], d.get('timed_pass_sclk_mhz'), d.get('timed_check_mismatches'), d.get('stencil_8192_MLUPS'), d.get('stencil_8192_sclk_mhz'), d.get('stencil_8192_check_mismatches'))"
done
echo R06L_OK
