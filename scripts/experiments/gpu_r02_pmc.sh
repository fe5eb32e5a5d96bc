#!/bin/bash
# Round-2 hardware-counter pass over the production configuration of every
# hot kernel (gmt_kernel_bench --only=hot,...): one rocprofv3 --pmc run per
# counter group (gfx950 slot limits: 8 SQ, 4 TCC, 2 GRBM per pass), plus a
# kernel trace (VGPR / SGPR / scratch per dispatch).  Counters that the box's
# rocprofv3 -L does not list are dropped from their group.
# Usage: scripts/gpu_r02_pmc.sh OUTDIR [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${1:-gpurun_out/pmc}
shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--only=hot,daxpy,stencil,pack --iters=3)
mkdir -p "$OUT"
BIN=$R/build/bin/gmt_kernel_bench
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || { echo "rocprofv3 -L failed"; tail -5 "$OUT/counters_list.txt"; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o kt -- "$BIN" "${ARGS[@]}" \
  > "$OUT/trace.log" 2>&1 || { echo "kernel trace failed"; tail -20 "$OUT/trace.log"; exit 1; }
echo TRACE_OK
have() { grep -qw "$1" "$OUT/counters_list.txt"; }
groups=(
  "FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"
  "WRITE_SIZE GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"
  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MFMA_F64 SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA TCC_HIT_sum TCC_MISS_sum"
  "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_FLAT SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
)
i=0
for g in "${groups[@]}"; do
  i=$((i + 1))
  sel=""
  for c in $g; do have "$c" && sel="$sel $c"; done
  echo "pass $i:$sel"
  [ -z "$sel" ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $sel --output-format csv -d "$OUT/pmc$i" -o p -- "$BIN" "${ARGS[@]}" \
    > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$OUT/pmc$i.log"; exit 1; }
done
echo PMC_OK
