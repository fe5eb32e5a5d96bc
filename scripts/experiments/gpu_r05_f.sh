#!/bin/bash
# Round 5 (f): the exec-masked Dirichlet keep + corner-only push fix.
#   (c) push numerics, TB bitwise tests, N = 8 shares, two ranks over IPC;
#   (d) Dirichlet rates new / head (per-cell select) / short, then bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash scripts/experiments/gpu_r05_c.sh && bash scripts/experiments/gpu_r05_d.sh
