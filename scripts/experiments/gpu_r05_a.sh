#!/bin/bash
# Round 5 (a): baseline of the K = 20 pass on this tree, and whether the
# unrolled bodies (27 KB per stage, 8 bodies in the kernel) miss in the
# instruction cache: sustained rates at mask 0 / 15, then rocprofv3 --pmc
# passes with the SQC instruction-cache counters for both masks.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r05_a}
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for m in 0 15 0 15; do
  for shp in "--jacobi-n=32768 --iters=20" "--jacobi-n=8192 --iters=200"; do
    timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=$m $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
  done
done
grep MLUPS $OUT/rates.log
cd /tmp
groups=(
  "GRBM_GUI_ACTIVE SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
  "GRBM_GUI_ACTIVE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
)
for m in 0 15; do
  i=0
  for g in "${groups[@]}"; do
    i=$((i + 1))
    echo "mask $m pass $i: $g"
    timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d "$OUT/pmc_m${m}_$i" -o p -- "$B" --only=tb --tb-k=20 --tb-mask=$m --jacobi-n=32768 --iters=3 \
      > "$OUT/pmc_m${m}_$i.log" 2>&1 || { echo "pmc pass $m $i failed"; tail -20 "$OUT/pmc_m${m}_$i.log"; exit 1; }
  done
done
echo PMC_OK
