#!/bin/bash
# Round 5 (k): host-staged exchange with the receive leg on its own stream;
# rank binding A/B for the slow mode; the push pass timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r05_k
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_gpu.py -k "host or stage or check" \
  "tests/test_kernels_gpu.py::test_stage_gather_scatter_field_blocks" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
M=/opt/conda/bin/mpirun
for rep in 1 2 3 4; do
  for bind in none core; do
    b=""; [ $bind = core ] && b="-bind-to core"
    timeout -k 10 120 $M -np 2 $b build/bin-host/mpi_halo_bench 8388608 8388608 30 --transport=mpi-direct > $OUT/alone_${bind}_$rep.txt 2>&1 || { tail $OUT/alone_${bind}_$rep.txt; exit 1; }
    mkdir -p $OUT/halo_${bind}_$rep
    GMT_HOST_TRACE=$OUT/halo_${bind}_$rep timeout -k 10 120 $M -np 2 $b build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_${bind}_$rep.txt 2>&1 || { tail $OUT/halo_${bind}_$rep.txt; exit 1; }
    timeout -k 10 120 $M -np 2 $b build/bin/mpi_stencil2d_sycl 1024 1 > $OUT/sycl_${bind}_$rep.txt 2>&1 || { tail $OUT/sycl_${bind}_$rep.txt; exit 1; }
    echo "rep $rep bind $bind: alone $(grep -E '^ *8388608' $OUT/alone_${bind}_$rep.txt | head -1) | mpi-host $(grep -E '^ *8388608' $OUT/halo_${bind}_$rep.txt | head -1) | sycl $(grep 'exchange time' $OUT/sycl_${bind}_$rep.txt | head -1)"
  done
done
B=$R/build/bin
for mode in "serial:--no-overlap" "push:--push"; do
  name=${mode%%:*}; opts=${mode#*:}
  timeout -k 10 180 $M -np 1 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$name -o $name -- \
    $B/mpi_jacobi2d 0 2000 --ny=8192 --nx=16384 --periodic --tblock --tsteps=20 --warmup=100 --transport=rccl $opts \
    > $OUT/prof_$name.log 2>&1 || { tail -20 $OUT/prof_$name.log; exit 1; }
  grep "TIME step" $OUT/prof_$name.log
done
echo R05K_OK
