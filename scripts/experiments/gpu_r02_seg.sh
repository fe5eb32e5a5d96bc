#!/bin/bash
# jacobi5tb numerics, then a segment-length / workgroup-width sweep at 32768^2
# and 8192^2 (Dirichlet on every side: rule waves at the edges included).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${1:-gpurun_out/seg}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_jacobi_tb_gpu.py -q -x --timeout 120 --timeout-method thread \
  > "$OUT/pytest_tb.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_tb.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
B=build/bin/gmt_kernel_bench
timeout -k 10 400 $B --only=hot,tb --hot-k=14 --iters=5 --tb-k=12,14,16 --tb-nw=4 --tb-seg=192,256,384,512,768,1024 \
  > "$OUT/kb_32768.log" 2>&1 || { tail -5 "$OUT/kb_32768.log"; exit 1; }
grep MLUPS "$OUT/kb_32768.log"
timeout -k 10 300 $B --only=hot,tb --hot-k=12 --iters=10 --jacobi-n=8192 --tb-k=10,12,14 --tb-nw=1,4 --tb-seg=96,128,192 \
  > "$OUT/kb_8192.log" 2>&1 || { tail -5 "$OUT/kb_8192.log"; exit 1; }
grep MLUPS "$OUT/kb_8192.log"
exit $rc
