#!/bin/bash
# Round 3: paired two-stage strips (build/var/pair: the two strips of a
# workgroup trade their inner edge columns through LDS, 464 output columns
# per 512 computed at K = 20 instead of 2 x 216): bitwise checks against the
# serial host run for every two-stage K, Dirichlet / periodic / band-first /
# 2 IPC ranks; then sustained K = 20 rates against the production kernel,
# alternating twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/r03_h}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
V=${V:-pair}
chk() {  # args...: run mpi_jacobi2d --check against the variant, require max|diff| == 0
  LD_LIBRARY_PATH=build/var/$V timeout -k 10 120 "$@" > $OUT/chk.log 2>&1 || { cat $OUT/chk.log; echo "FAILED: $*"; exit 1; }
  d=$(grep -oE "vs serial = [0-9.e+-]+" $OUT/chk.log | awk '{print $4}')
  echo "$d  $*" | tee -a $OUT/checks.txt
  python3 -c "import sys; sys.exit(0 if float('$d') == 0.0 else 1)" || { cat $OUT/chk.log; echo "NOT BITWISE: $*"; exit 1; }
}
: > $OUT/checks.txt
for k in 12 14 16 18 20; do
  chk build/bin/mpi_jacobi2d --ny=700 --nx=1900 0 47 --check --tblock --tsteps=$k
  chk build/bin/mpi_jacobi2d --ny=700 --nx=1900 0 47 --check --tblock --tsteps=$k --periodic
done
chk build/bin/mpi_jacobi2d --ny=333 --nx=517 0 41 --check --tblock --tsteps=20
chk build/bin/mpi_jacobi2d --ny=1500 --nx=1900 0 47 --check --tblock --tsteps=20 --periodic --transport=rccl --overlap
chk build/bin/mpi_jacobi2d --ny=1500 --nx=1900 0 47 --check --tblock --tsteps=20 --periodic=x --transport=rccl --overlap
chk $M -np 2 build/bin/mpi_jacobi2d --ny=701 --nx=1900 0 47 --check --tblock --tsteps=20 --transport=ipc --dims=2x1
chk $M -np 2 build/bin/mpi_jacobi2d --ny=701 --nx=1900 0 47 --check --tblock --tsteps=20 --transport=ipc --dims=1x2
B=build/bin/gmt_kernel_bench
for rep in 1 2; do
  for v in base $V; do
    lp=""; [ "$v" != base ] && lp=build/var/$v
    : > $OUT/$v.$rep.log
    for shp in "--jacobi-n=32768 --iters=20" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=100" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=100" "--jacobi-n=8192 --iters=100"; do
      LD_LIBRARY_PATH=$lp timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/$v.$rep.log 2>&1 || { cat $OUT/$v.$rep.log; exit 1; }
    done
    echo "$v: $(grep MLUPS $OUT/$v.$rep.log | awk '{print $(NF-13)}' | tr '\n' ' ')"
  done
done
