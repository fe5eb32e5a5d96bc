#!/bin/bash
# Round 4 (bb): the driver's N = 8 launch shape rehearsed on the one-GPU box:
# 8 ranks sharing cuda:0 (IPC), transport probe on (8 probe children, then
# the 8 ranks), the full bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_bb}
mkdir -p $OUT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 8 --steps 20 --warmup 5 --transport-probe on \
  > $OUT/bench_n8.json 2> $OUT/bench_n8.err || { tail -40 $OUT/bench_n8.err; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$OUT/bench_n8.json') if l.startswith('{')][0]); print(r['value'], r['config']['parallelism'], r['config']['transport'], r.get('transport_candidates'), r.get('transport_probe_s'), r['check_max_diff'], r['stencil_alt_dims'], r['ref_halo_dim0_bad_ghosts'], r['daxpy_allsum_rel_err'])"
