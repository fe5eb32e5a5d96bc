#!/bin/bash
# Pipelined Jacobi with the rule bands split off: numerics, kernel A/B, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/split${TAG:-}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "jacobi5xk" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
M=/opt/conda/bin/mpirun
timeout -k 10 120 $M -np 1 build/bin/mpi_jacobi2d 515 30 --check --periodic --graph --transport=rccl --tblock --tsteps=8 --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
grep -E "check" $OUT/jc.log
timeout -k 10 120 $M -np 4 build/bin/mpi_jacobi2d 515 30 --check --tblock --tsteps=8 --dims=2x2 --periodic --transport=ipc --warmup=3 > $OUT/jc.log 2>&1 || { cat $OUT/jc.log; exit 1; }
grep -E "check" $OUT/jc.log
timeout -k 10 400 build/bin/gmt_kernel_bench --iters=10 --only=jacobi --sections=pipe --jacobi-n=32768 > $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
timeout -k 10 200 build/bin/gmt_kernel_bench --iters=20 --only=jacobi --sections=pipe --jacobi-n=8192 >> $OUT/kb.log 2>&1 || { cat $OUT/kb.log; exit 1; }
grep -E "pipe" $OUT/kb.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 16 --warmup 0 --graph off --skip-extras > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
echo PROF_OK
