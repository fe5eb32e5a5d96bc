#!/bin/bash
# strong-scaling shares + hardware counters of the round-2 hot kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/shares
./scripts/gpu_r02_shares.sh > gpurun_out/shares/shares.txt 2>&1 || { tail -20 gpurun_out/shares/shares.txt; exit 1; }
cat gpurun_out/shares/shares.txt
scripts/gpu_r02_pmc.sh gpurun_out/pmc6 --only=hot,stencil --hot-k=12,20 --iters=3 || exit 1
