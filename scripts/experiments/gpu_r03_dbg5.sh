#!/bin/bash
# Round 3 debug: 2 ranks, y split (2x1), K = 20, serial — which layer goes stale?
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export GMT_TEST_DEVICE=cuda OMP_NUM_THREADS=1 GMT_TEST_GRAPH=0
run() {  # np ny nx steps periodic overlap tblock dims [env...]
  local np=$1; shift
  timeout -k 10 120 env "${@:8}" python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $((20000 + RANDOM % 20000)) tests/engine_mp_worker.py "${@:1:7}" 2>/dev/null | grep '^{' | cut -c1-150 || echo "FAILED rc=$?"
}
app() { timeout -k 10 120 /opt/conda/bin/mpirun -np 2 build/bin/mpi_jacobi2d --ny=313 --nx=1695 0 "$@" 2>&1 | grep -E "check|transport|ERROR|error" | head -3; }
echo "a1 engine ipc 2x1 K20 43: $(run 2 313 1695 43 0 0 20 2x1)"
echo "a2 engine ipc 2x1 K20 43: $(run 2 313 1695 43 0 0 20 2x1)"
echo "b  serialized kernels:     $(run 2 313 1695 43 0 0 20 2x1 AMD_SERIALIZE_KERNEL=3)"
echo "e1 steps 20:               $(run 2 313 1695 20 0 0 20 2x1)"
echo "e2 steps 40:               $(run 2 313 1695 40 0 0 20 2x1)"
echo "f1 K18:                    $(run 2 313 1695 43 0 0 18 2x1)"
echo "f2 K16:                    $(run 2 313 1695 43 0 0 16 2x1)"
echo "f3 K10:                    $(run 2 313 1695 43 0 0 10 2x1)"
echo "g  periodic 1 rank K20:    $(run 1 313 1695 43 1 0 20 1x1)"
echo "c  app mpi-host 2x1 K20:"; app 43 --check --tblock --tsteps=20 --no-overlap --dims=2x1 --transport=mpi-host
echo "d  app ipc 2x1 K20:"; app 43 --check --tblock --tsteps=20 --no-overlap --dims=2x1 --transport=ipc
echo "d2 app ipc 1x2 K20:"; app 43 --check --tblock --tsteps=20 --no-overlap --dims=1x2 --transport=ipc
