set -o pipefail
mkdir -p gpurun_out/r2g
B=build/bin/gmt_kernel_bench
timeout -k 10 300 $B --only=tb --iters=5 --tb-k=12,14 --tb-nw=1,4 --tb-p=3 --tb-seg=0,256,512,1024 > gpurun_out/r2g/seg.log 2>&1 || exit 1
grep MLUPS gpurun_out/r2g/seg.log
LD_LIBRARY_PATH=$PWD/build/exp timeout -k 10 300 $B --only=tb --iters=5 --tb-k=12,14 --tb-nw=2,4,8 --tb-p=3 > gpurun_out/r2g/nobar.log 2>&1 || exit 1
echo "== no barrier (timing only, results invalid)"
grep MLUPS gpurun_out/r2g/nobar.log
