#!/bin/bash
# kernel trace of bench.py (1 GPU, driver config) with the 3-column kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4/raw -o bench -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof4/bench.json 2> gpurun_out/prof4/bench.err
rc=$?
find gpurun_out/prof4/raw -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof4/kernel_stats.csv \;
find gpurun_out/prof4/raw -name "*kernel_trace.csv" -exec cp {} gpurun_out/prof4/kernel_trace.csv \;
rm -rf gpurun_out/prof4/raw
exit $rc
