#!/bin/bash
# Round 4 (c): why the wide K = 20 kernel loses.  Sustained rates of the
# production (wide) kernel against diagnostic variants with no step barrier
# (nobar) and no DPP lane shifts (nodpp) — both give wrong results, they
# bound what those costs are — and the round-3 kernel; then rocprofv3 --pmc
# passes on the round-3 and the wide kernel (32768^2, K = 20, 3 passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_c}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
for v in r03 new nobar nodpp; do
  lp=""; [ "$v" != new ] && lp=$R/build/ab_$v
  : > $OUT/$v.log
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100"; do
    LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/$v.log 2>&1 || { cat $OUT/$v.log; exit 1; }
  done
  echo "$v: $(grep MLUPS $OUT/$v.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
done
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || echo "rocprofv3 -L failed"
have() { grep -qw "$1" "$OUT/counters_list.txt"; }
groups=(
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
  "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_ADD_F64 SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS"
)
for v in r03 new; do
  lp=""; [ "$v" != new ] && lp=$R/build/ab_$v
  i=0
  for g in "${groups[@]}"; do
    i=$((i + 1))
    sel=""; n=0
    for c in $g; do have "$c" && { sel="$sel $c"; n=$((n + 1)); }; done
    echo "$v pass $i:$sel"
    LD_LIBRARY_PATH=$lp timeout -s KILL 120 rocprofv3 --pmc $sel --output-format csv -d "$OUT/pmc_${v}_$i" -o p -- "$B" --only=tb --tb-k=20 --tb-mask=0 --jacobi-n=32768 --iters=3 \
      > "$OUT/pmc_${v}_$i.log" 2>&1 || { echo "pmc pass $v $i failed"; tail -20 "$OUT/pmc_${v}_$i.log"; exit 1; }
  done
done
echo PMC_OK
