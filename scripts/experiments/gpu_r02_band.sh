#!/bin/bash
# band-first overlap: GPU tests, then the strong-scaling shares (serial /
# overlapped / auto) on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/band
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_gpu.py \
  -k "band_first or periodic_matches or dirichlet_repeated or autotune or ipc_graph or jacobi_check" \
  > gpurun_out/band/pytest.log 2>&1 || { tail -40 gpurun_out/band/pytest.log; exit 1; }
tail -3 gpurun_out/band/pytest.log
OUT=gpurun_out/band bash scripts/gpu_r02_shares.sh
