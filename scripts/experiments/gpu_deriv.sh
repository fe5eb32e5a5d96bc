#!/bin/bash
# dim-1 derivative window variants: numerics + timing at the reference shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/deriv
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "stencil" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 build/bin/gmt_kernel_bench --iters=20 --only=stencil > $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
cat $OUT/kb.log
