#!/bin/bash
# VALU issue-rate microbenchmark (csrc/bench/valu_rate.hip) + its clock, and
# counters of the temporal-blocking kernel at K = 14 / 16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${1:-gpurun_out/valu}
mkdir -p "$OUT"
R=$PWD
timeout -k 10 120 build/bench/valu_rate 20000 > "$OUT/valu_rate.txt" 2>&1 || { cat "$OUT/valu_rate.txt"; exit 1; }
cat "$OUT/valu_rate.txt"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES \
  --output-format csv -d "$R/$OUT/pmc_valu" -o p -- "$R/build/bench/valu_rate" 5000 > "$R/$OUT/pmc_valu.log" 2>&1 || { tail "$R/$OUT/pmc_valu.log"; exit 1; }
cd "$R"
scripts/gpu_r02_pmc.sh "$OUT/pmc_tb" --only=tb --tb-k=14,16 --tb-nw=1 --tb-p=6 --iters=2 || exit 1
