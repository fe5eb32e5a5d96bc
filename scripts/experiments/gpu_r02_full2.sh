#!/bin/bash
# full GPU suite + smoke + bench + kernel trace, then the transport numbers
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
./scripts/gpu_r02_full.sh ${1:-gpurun_out/full5} && ./scripts/gpu_r02_xport.sh ${2:-gpurun_out/xport}
