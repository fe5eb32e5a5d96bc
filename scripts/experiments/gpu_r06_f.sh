#!/bin/bash
# Round 6 (f): ten default (unbound, self-pinned) launches of the host-staged
# 8 MiB exchange at 2 ranks — the verdict's done-means for rank pinning.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_f
mkdir -p $OUT
M=/opt/conda/bin/mpirun
: > $OUT/pin10.txt
for rep in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 120 $M -np 2 build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_$rep.txt 2>&1 || { tail $OUT/halo_$rep.txt; exit 1; }
  echo "rep $rep: $(grep 'pinned cpu' $OUT/halo_$rep.txt) | $(grep -E '^ *8388608' $OUT/halo_$rep.txt | head -1)" | tee -a $OUT/pin10.txt
done
echo R06F_OK
