#!/bin/bash
# Round 6 (b): the clock record — cost A/B (GMT_CLOCK=0), the clock per timed
# run at 32768^2 and 8192^2, three driver-config bench runs on one box (does
# MLUPS track timed_pass_sclk_mhz?), and the new kernel GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_push_gpu.py tests/test_production_geometry_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u scripts/experiments/clock_ab.py 32768 20 6 > $OUT/clock_ab_32768.txt 2>&1 || { tail -20 $OUT/clock_ab_32768.txt; exit 1; }
cat $OUT/clock_ab_32768.txt | grep "^n "
timeout -k 10 200 python -u scripts/experiments/clock_ab.py 8192 1000 6 > $OUT/clock_ab_8192.txt 2>&1 || { tail -20 $OUT/clock_ab_8192.txt; exit 1; }
cat $OUT/clock_ab_8192.txt | grep "^n "
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$rep.out 2> $OUT/bench_$rep.err || { tail -30 $OUT/bench_$rep.err; exit 1; }
  tail -1 $OUT/bench_$rep.out > $OUT/bench_$rep.json
  python3 -c "
import json; d = json.load(open('$OUT/bench_$rep.json'))
print('bench $rep', d['value'], d['timed_pass_sclk_mhz'], d['timed_pass_clock_samples'], d['timed_check_mismatches'], d.get('stencil_8192_MLUPS'), d.get('stencil_8192_sclk_mhz'))"
done
# rank pinning (default on): 10 unbound launches of the host-staged 8 MiB
# exchange at 2 ranks, then 4 with GMT_PIN=0 (A/B), and the reference's
# stage_host exchange (mpi_stencil2d_sycl 1024 1)
M=/opt/conda/bin/mpirun
: > $OUT/pin_rates.txt
for rep in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 120 $M -np 2 build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_pin_$rep.txt 2>&1 || { tail $OUT/halo_pin_$rep.txt; exit 1; }
  echo "pin rep $rep: $(grep -E '^ *8388608' $OUT/halo_pin_$rep.txt | head -1)" | tee -a $OUT/pin_rates.txt
done
for rep in 1 2 3 4; do
  GMT_PIN=0 timeout -k 10 120 $M -np 2 build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_nopin_$rep.txt 2>&1 || { tail $OUT/halo_nopin_$rep.txt; exit 1; }
  echo "GMT_PIN=0 rep $rep: $(grep -E '^ *8388608' $OUT/halo_nopin_$rep.txt | head -1)" | tee -a $OUT/pin_rates.txt
done
for rep in 1 2 3; do
  timeout -k 10 120 $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 > $OUT/sycl_$rep.txt 2>&1 || { tail $OUT/sycl_$rep.txt; exit 1; }
  echo "sycl 1024 1 rep $rep: $(grep 'exchange time' $OUT/sycl_$rep.txt | tr '\n' ' ')" | tee -a $OUT/pin_rates.txt
done
timeout -k 10 120 $M -np 2 build/bin/mpi_stencil2d_gt 256 20 --n-other=65536 --debug > $OUT/gt_debug.txt 2>&1 || { tail $OUT/gt_debug.txt; exit 1; }
grep -E "exchange time|err_norm|allreduce time" $OUT/gt_debug.txt | head -6
echo R06B_OK
