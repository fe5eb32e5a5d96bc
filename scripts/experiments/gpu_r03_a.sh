#!/bin/bash
# Round 3, first GPU pass: multi-rank (oversubscribed, IPC) bench path, the
# IPC app tests after the kernel rewrite, and the driver-config bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r03_a
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 480 --timeout-method thread -m gpu \
  tests/test_multirank_gpu.py "tests/test_native_gpu.py::test_app_jacobi_ipc_graph_matches_serial" \
  "tests/test_native_gpu.py::test_app_ipc_halo_latency" "tests/test_native_gpu.py::test_app_jacobi_band_first" \
  > $OUT/pytest.log 2>&1; rc=$?
tail -30 $OUT/pytest.log
exit $rc
