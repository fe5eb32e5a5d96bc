#!/bin/bash
# Round 6 (aa): two-strip shared hand-off groups (Sh<K, 2>: 448 output
# columns per 4 waves at K = 20) — bitwise tests, then same box,
# alternating: the defaults (nw2 = two stage-major strips for large
# Dirichlet passes / one strip), sh2 (GMT_TB_SHARED=2), sh4 (=4).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_aa
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_tb_shared_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in 1 2; do
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=32768 --iters=20"; do
    for mask in 0 15; do
      for v in def sh2 sh4; do
        case $v in
          def) envs="GMT_TB_SHARED=0";;
          sh2) envs="GMT_TB_SHARED=2";;
          sh4) envs="GMT_TB_SHARED=4";;
        esac
        echo "== $v m$mask $shp" >> $OUT/rates.log
        env $envs timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$mask $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
      done
    done
  done
done
grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $5, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
echo R06AA_OK
