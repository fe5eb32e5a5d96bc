#!/bin/bash
# Per-pass cost of the temporal-blocking kernel for every K (defaults), at
# 32768^2 and 8192^2, and bench.py at 8192^2 for K = 10, 12, 14.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${1:-gpurun_out/costs}
mkdir -p "$OUT"
B=build/bin/gmt_kernel_bench
timeout -k 10 300 $B --only=tb --iters=7 --tb-k=2,4,6,8,10,12,14,16 --tb-nw=4 > "$OUT/kb_32768.log" 2>&1 || { tail -5 "$OUT/kb_32768.log"; exit 1; }
grep "ms" "$OUT/kb_32768.log"
timeout -k 10 300 $B --only=tb --iters=15 --jacobi-n=8192 --tb-k=2,4,6,8,10,12,14,16 --tb-nw=4 > "$OUT/kb_8192.log" 2>&1 || { tail -5 "$OUT/kb_8192.log"; exit 1; }
grep "ms" "$OUT/kb_8192.log"
for k in 10 12 14; do
  timeout -k 10 200 python bench.py --size 8192 --steps 400 --warmup 20 --tsteps $k --skip-extras --skip-check > "$OUT/b8192_k$k.json" 2>> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b8192_k$k.json'));print($k, d['value'], d['config']['pass_plan'])"
done
