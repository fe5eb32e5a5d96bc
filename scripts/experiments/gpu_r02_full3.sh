#!/bin/bash
# full GPU suite + smoke + bench + kernel trace, then the strong-scaling shares
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
./scripts/gpu_r02_full.sh ${1:-gpurun_out/full6} && mkdir -p gpurun_out/shares && ./scripts/gpu_r02_shares.sh > gpurun_out/shares/shares.txt 2>&1 && cat gpurun_out/shares/shares.txt
