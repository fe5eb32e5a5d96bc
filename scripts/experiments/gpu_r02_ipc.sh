#!/bin/bash
# stream-ordered IPC: native GPU tests, then latency / bandwidth numbers
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/ipc
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_native_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/ipc/tests.log 2>&1 || { tail -40 gpurun_out/ipc/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/ipc/tests.log | tail -25
M=/opt/conda/bin/mpirun
timeout -k 10 120 $M -np 2 build/bin/mpi_halo_bench 16 16777216 30 --transport=ipc > gpurun_out/ipc/halo_ipc2.log 2>&1 && cat gpurun_out/ipc/halo_ipc2.log | tail -25
