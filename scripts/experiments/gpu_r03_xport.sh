#!/bin/bash
# Round 3: host-staged transport, kernel-driven D2H staging (GMT_HOST_STAGE=kernel,
# default) vs the round-2 SDMA chunks (sdma), 2 ranks on one GPU; the
# reference's stage_host exchange; IPC latency after the table-driven kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${1:-gpurun_out/r03_xport}
mkdir -p $OUT
M=/opt/conda/bin/mpirun
run() { local t=$1 name=$2; shift 2; echo "=== $name: $*" >> $OUT/summary.txt; timeout -k 10 $t "$@" >> $OUT/summary.txt 2>&1 || { echo "FAILED $name rc=$?"; tail -20 $OUT/summary.txt; exit 1; }; }
: > $OUT/summary.txt
for rep in 1 2; do
GMT_HOST_STAGE=kernel run 120 halo_host_kernel_$rep $M -np 2 build/bin/mpi_halo_bench 65536 16777216 20 --transport=mpi-host
GMT_HOST_STAGE=sdma run 120 halo_host_sdma_$rep $M -np 2 build/bin/mpi_halo_bench 65536 16777216 20 --transport=mpi-host
GMT_HOST_STAGE=kernel run 120 sycl_stage1_kernel_$rep $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50
GMT_HOST_STAGE=sdma run 120 sycl_stage1_sdma_$rep $M -np 2 build/bin/mpi_stencil2d_sycl 1024 1 50
done
run 120 halo_ipc2 $M -np 2 build/bin/mpi_halo_bench 16 1024 200 --transport=ipc
run 120 host_mpi_ceiling $M -np 2 build/bin-host/mpi_halo_bench 65536 16777216 20 --transport=mpi-direct
grep -E "^ +[0-9]+ +2 |exchange time|===" $OUT/summary.txt
# oversubscribed bench at 2 ranks: the IPC all-reduces (residual, DAXPY partial sums, 1024-double test_sum)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --size 8192 --steps 20 --warmup 5 --daxpy-n 16777216 --ref-iters 20 > $OUT/bench_n2.json 2> $OUT/bench_n2.err &&
python -c "import json;d=json.load(open('$OUT/bench_n2.json'));print({k:d[k] for k in ('value','check_max_diff','daxpy_allreduce_us','ref_allreduce_1024_us','daxpy_allsum_rel_err','halo_exchange_us','ref_halo_dim0_us','ref_halo_dim1_us')})"
