#!/bin/bash
# Round 4 (e): wide K = 20 kernel diagnostics after the lag-3 hand-off:
# DMA depth P = 5 / 9 (runtime ring slots), no sched_barrier between levels
# (nosb), no step barrier (nobar, wrong results: a bound), vs production and
# round 3; then the counters of the production kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_e}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
for rep in 1 2; do
  for v in r03 new p5 p9 nosb nobar; do
    lp=""; [ "$v" != new ] && lp=$R/build/ab_$v
    : > $OUT/$v.$rep.log
    for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100"; do
      LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/$v.$rep.log 2>&1 || { cat $OUT/$v.$rep.log; exit 1; }
    done
    echo "$v: $(grep MLUPS $OUT/$v.$rep.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
  done
done
cd /tmp
groups=(
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
  "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_ADD_F64 SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS"
)
i=0
for g in "${groups[@]}"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/pmc_new_$i" -o p -- "$B" --only=tb --tb-k=20 --tb-mask=0 --jacobi-n=32768 --iters=3 \
    > "$OUT/pmc_new_$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$OUT/pmc_new_$i.log"; exit 1; }
done
echo PMC_OK
# host-staged exchange: halo faces staged in place (default) vs packed through
# device buffers (GMT_HOST_BLOCKS=0, the round-3 path), 2 ranks on one GPU
cd $R
M=/opt/conda/bin/mpirun
run() { local t=$1 name=$2; shift 2; echo "=== $name: $*" >> $OUT/xport.txt; timeout -k 10 $t "$@" >> $OUT/xport.txt 2>&1 || { echo "FAILED $name rc=$?"; tail -20 $OUT/xport.txt; exit 1; }; }
: > $OUT/xport.txt
for rep in 1 2; do
  run 120 sycl_blocks_$rep $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50
  GMT_HOST_BLOCKS=0 run 120 sycl_packed_$rep $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50
  run 120 halo_blocks_$rep $M -np 2 build/bin/mpi_halo_bench 65536 16777216 20 --transport=mpi-host
  GMT_HOST_BLOCKS=0 run 120 halo_packed_$rep $M -np 2 build/bin/mpi_halo_bench 65536 16777216 20 --transport=mpi-host
done
grep -E "^ +[0-9]+ +2 |exchange time|===" $OUT/xport.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_native_gpu.py -k "halo_check or stencil2d_gt_err or jacobi_check" > $OUT/pytest_xport.log 2>&1 || { tail -30 $OUT/pytest_xport.log; exit 1; }
tail -2 $OUT/pytest_xport.log
