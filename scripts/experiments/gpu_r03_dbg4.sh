#!/bin/bash
# Round 3 debug: 4 oversubscribed ranks (2x2, IPC) vs the serial reference,
# overlap on/off, one- and two-phase corners, a few K.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export GMT_TEST_DEVICE=cuda OMP_NUM_THREADS=1
run() {  # np ny nx steps periodic overlap tblock dims [env...]
  local np=$1; shift
  timeout -k 10 120 env "${@:8}" python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $((20000 + RANDOM % 20000)) tests/engine_mp_worker.py "${@:1:7}" 2>/dev/null | grep '^{' || echo "FAILED rc=$?"
}
for tp in 0 1; do for ov in 0 1; do for k in 4 12 20; do
  echo "two_phase=$tp overlap=$ov K=$k: $(run 4 313 1695 43 0 $ov $k 2x2 GMT_HALO_TWO_PHASE=$tp GMT_TEST_GRAPH=0)"
done; done; done
echo "1x4 overlap=1 K=20: $(run 4 313 3000 43 0 1 20 1x4 GMT_TEST_GRAPH=0)"
echo "4x1 overlap=1 K=20: $(run 4 700 900 43 0 1 20 4x1 GMT_TEST_GRAPH=0)"
echo "2x1 overlap=0 K=20: $(run 2 313 1695 43 0 0 20 2x1 GMT_TEST_GRAPH=0)"
echo "1x2 overlap=0 K=20: $(run 2 313 1695 43 0 0 20 1x2 GMT_TEST_GRAPH=0)"
echo "2x2 periodic overlap=0 K=4: $(run 4 100 140 9 1 0 4 2x2 GMT_TEST_GRAPH=0)"
echo "2x2 overlap=0 K=1: $(run 4 100 140 9 0 0 0 2x2 GMT_TEST_GRAPH=0)"
