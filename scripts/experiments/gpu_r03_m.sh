#!/bin/bash
# Round 3: IPC exchange with one system fence per workgroup: IPC GPU tests
# (bitwise), then the 16-B latency (2 ranks on one GPU), three runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r03_m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_native_gpu.py \
  tests/test_multirank_gpu.py -k "ipc or IPC or oversubscribed or hang or band_first" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc = 0 ] || { grep -B5 -A30 FAILURES $OUT/pytest.log | head -60; exit $rc; }
for r in 1 2 3; do
  timeout -k 10 120 /opt/conda/bin/mpirun -np 2 build/bin/mpi_halo_bench 16 4096 200 --transport=ipc > $OUT/lat$r.txt 2>&1 || { cat $OUT/lat$r.txt; exit 1; }
  grep -E "^\s+16\s" $OUT/lat$r.txt
done
