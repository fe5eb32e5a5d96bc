#!/bin/bash
# Round 4 (i): conflict-free piece-major LDS rows (production) vs the
# row-ordered layout (build/ab_base = HEAD before it), narrow K = 20, and the
# wide kernel with the same layout (build/ab_wide); bitwise tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_i}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_jacobi_tb_gpu.py tests/test_native_gpu.py tests/test_multirank_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A40 FAILURES $OUT/pytest.log | head -80; exit $rc; }
LD_LIBRARY_PATH=$R/build/ab_wide timeout -k 10 120 build/bin/mpi_jacobi2d --ny=700 --nx=1900 0 47 --check --tblock --tsteps=20 2>&1 | grep -E "vs serial" | tee $OUT/wide_check.txt
B=$R/build/bin/gmt_kernel_bench
for rep in 1 2 3; do
  for v in base new wide; do
    lp=""; [ "$v" != new ] && lp=$R/build/ab_$v
    : > $OUT/$v.$rep.log
    for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=100" "--jacobi-n=8192 --iters=100"; do
      LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/$v.$rep.log 2>&1 || { cat $OUT/$v.$rep.log; exit 1; }
    done
    echo "$v: $(grep MLUPS $OUT/$v.$rep.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
  done
done
cd /tmp
for v in base new; do
  lp=""; [ "$v" != new ] && lp=$R/build/ab_$v
  LD_LIBRARY_PATH=$lp timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY \
    --output-format csv -d "$OUT/pmc_$v" -o p -- "$B" --only=tb --tb-k=20 --tb-mask=0 --jacobi-n=32768 --iters=3 > "$OUT/pmc_$v.log" 2>&1 || { echo "pmc $v failed"; tail -5 "$OUT/pmc_$v.log"; }
done
echo done
