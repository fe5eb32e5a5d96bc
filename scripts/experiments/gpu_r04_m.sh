#!/bin/bash
# Round 4 (m): band-first with the column-band-aware planner (bands done by
# ~70% of the pass) + the exchange's pack/unpack as a few-workgroup
# grid-stride copy (Halo2D::set_pack_wgs, 128 by default) vs HEAD
# (build/ab_head, full-grid pack: GMT_PACK_WGS=0); serial vs overlap on the N = 8 shares, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_m}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_jacobi_tb_gpu.py tests/test_native_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A40 FAILURES $OUT/pytest.log | head -80; exit $rc; }
: > $OUT/shares.txt
for rep in 1 2 3; do
  for cfg in "8192 16384" "16384 8192" "16384 16384"; do
    set -- $cfg
    for v in head new new64 new0; do
      lp=""; [ "$v" = head ] && lp=$R/build/ab_head
      pw=""; [ "$v" = new64 ] && pw=64; [ "$v" = new0 -o "$v" = head ] && pw=0
      for mode in "--no-overlap" "--overlap"; do
        [ "$mode" = "--no-overlap" ] && [ "$v" = new64 -o "$v" = new0 ] && continue
        env ${pw:+GMT_PACK_WGS=$pw} LD_LIBRARY_PATH=$lp timeout -k 10 200 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 --graph \
          --periodic --transport=rccl $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
        echo "rep=$rep $v ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log)" | tee -a $OUT/shares.txt
      done
    done
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- \
  build/bin/mpi_jacobi2d --ny=8192 --nx=16384 200 --tblock --tsteps=20 --warmup=20 \
  --periodic --transport=rccl --overlap > $OUT/tr.log 2>&1 || { tail -20 $OUT/tr.log; exit 1; }
grep "TIME step" $OUT/tr.log
