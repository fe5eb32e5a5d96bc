#!/bin/bash
# Round 3: W/E signalling bands of band-first passes: 3/4 of the segment
# length (build/var/lb34), or full length in multi-round launches and 3/4
# in single-round ones (build/var/lbad), vs L/3 (production): bitwise
# band-first checks, then the five shares
# (periodic, all four faces), serial vs band-first, alternating twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/r03_g}
mkdir -p $OUT
for p in "--periodic" "--periodic=x"; do
  for v in lb34 lbad; do
  LD_LIBRARY_PATH=build/var/$v timeout -k 10 120 build/bin/mpi_jacobi2d --ny=1500 --nx=1900 0 47 --check --tblock --tsteps=20 \
    $p --transport=rccl --overlap 2>&1 | grep -E "check|overlap" || { echo "$v check $p failed"; exit 1; }
  done
done
: > $OUT/shares.txt
for rep in 1 2; do
  for cfg in "32768 32768" "16384 32768" "16384 16384" "8192 16384" "16384 8192"; do
    set -- $cfg
    for v in base lb34 lbad; do
      lp=""; [ "$v" != base ] && lp=build/var/$v
      for mode in "--no-overlap" "--overlap"; do
        [ "$v" != base ] && [ "$mode" = "--no-overlap" ] && continue
        LD_LIBRARY_PATH=$lp timeout -k 10 200 build/bin/mpi_jacobi2d --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 --graph \
          --periodic --transport=rccl $mode > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
        echo "rep=$rep ny=$1 nx=$2 $v [$mode] $(grep -E 'TIME step' $OUT/j.log)" | tee -a $OUT/shares.txt
      done
    done
  done
done
