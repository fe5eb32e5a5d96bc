#!/bin/bash
# BASELINE single-GPU config 8192^2: bench at K = 8/12/14 + kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/b8192
mkdir -p $OUT
for K in 8 12 14; do
  timeout -k 10 300 python bench.py --size 8192 --steps 500 --warmup 20 --tsteps $K --skip-extras > $OUT/bench$K.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  echo "K=$K $(python3 -c "import json; r=json.load(open('$OUT/bench$K.json')); print(r['value'], r['ms_per_step'])")"
done
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/p -o b -- python3 $R/bench.py --size 8192 --steps 100 --warmup 14 --skip-extras > $R/$OUT/prof.json 2> $R/$OUT/prof.err || { tail -20 $R/$OUT/prof.err; exit 1; }
echo PROF_OK
