#!/bin/bash
# Round 3: band-first passes with the exchange on reserved CUs
# (GMT_COMM_CUS, CU-masked streams): bitwise engine/app tests, then the
# shares (periodic RCCL self-exchange) and the 1-rank host-staged exchange,
# serial vs band-first with 0 / 8 / 16 reserved CUs, two repetitions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$PWD
OUT=$R/gpurun_out/r03_l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_native_gpu.py tests/test_multirank_gpu.py tests/test_jacobi_tb_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A30 FAILURES $OUT/pytest.log | head -60; exit $rc; }
J=build/bin/mpi_jacobi2d
: > $OUT/ab.txt
run() {  # label env... -- args
  local label=$1; shift
  timeout -k 10 200 env "$@" > $OUT/j.log 2>&1 || { cat $OUT/j.log; exit 1; }
  echo "$label $(grep -E 'TIME step' $OUT/j.log)" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  for cfg in "8192 16384" "16384 8192" "16384 16384"; do
    set -- $cfg
    A="$J --ny=$1 --nx=$2 100 --tblock --tsteps=20 --warmup=20 --periodic --transport=rccl"
    run "rep=$rep $1x$2 serial" GMT_COMM_CUS=0 $A --no-overlap
    run "rep=$rep $1x$2 band cus=0" GMT_COMM_CUS=0 $A --overlap
    run "rep=$rep $1x$2 band cus=8" GMT_COMM_CUS=8 $A --overlap
    run "rep=$rep $1x$2 band cus=16" GMT_COMM_CUS=16 $A --overlap
  done
  A="$J 16384 100 --tblock --tsteps=20 --warmup=20 --periodic --transport=mpi-host"
  run "rep=$rep mpihost16384 serial" GMT_COMM_CUS=0 $A --no-overlap
  run "rep=$rep mpihost16384 band cus=0" GMT_COMM_CUS=0 $A --overlap
  run "rep=$rep mpihost16384 band cus=8" GMT_COMM_CUS=8 $A --overlap
  run "rep=$rep mpihost16384 band cus=16" GMT_COMM_CUS=16 $A --overlap
done
