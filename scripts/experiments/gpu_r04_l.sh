#!/bin/bash
# Round 4 (l): the exchange's pack/unpack as a grid-stride copy over few
# workgroups (GMT_PACK_WGS) so it fits the free slots beside a band-first
# pass: overlap vs serial on the N = 8 shares, and a kernel trace at 64.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_l}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "copy2d or halo" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A40 FAILURES $OUT/pytest.log | head -80; exit $rc; }
: > $OUT/shares.txt
for rep in 1 2; do
  for cfg in "8192 16384" "16384 8192"; do
    set -- $cfg
    for cap in 0 16 64 256; do
      for mode in "--no-overlap" "--overlap"; do
        GMT_PACK_WGS=$cap timeout -k 10 200 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 --graph \
          --periodic --transport=rccl $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
        echo "rep=$rep cap=$cap ny=$1 nx=$2 [$mode] $(grep -E 'TIME step' $OUT/j.log)" | tee -a $OUT/shares.txt
      done
    done
  done
done
GMT_PACK_WGS=64 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr64 -o tr -- \
  build/bin/mpi_jacobi2d --ny=8192 --nx=16384 200 --tblock --tsteps=20 --warmup=20 \
  --periodic --transport=rccl --overlap > $OUT/tr64.log 2>&1 || { tail -20 $OUT/tr64.log; exit 1; }
grep "TIME step" $OUT/tr64.log
