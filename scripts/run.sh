#!/bin/bash
# run.sh um|noum rocprof|none nodes ppn — distributed DAXPY + all-gather job.
#
# MI355X version of the reference launch script (/root/reference/summit/run.sh,
# jlse/run.sh): mpirun instead of jsrun, rocprofv3 instead of nsys/nvprof.
# With "rocprof" every rank writes its own trace directory; the roctx
# capture window (gmt_profiler_start/stop = the reference's
# cudaProfilerStart/Stop) limits collection to the benchmark body.
# Output: out-<tag>.txt (feed to scripts/avg.sh), profiles under profile/<tag>/.
set -u
if [ $# -ne 4 ]; then
  echo "Usage: $0 um|noum rocprof|none nodes ppn"
  exit 1
fi
um=$1 prof=$2 nodes=$3 ppn=$4
tag=${um}_${prof}_${nodes}_${ppn}
here=$(cd "$(dirname "$0")/.." && pwd)
bin=${GMT_BIN:-$here/build/bin}
mpirun=${MPIRUN:-/opt/conda/bin/mpirun}
# one core per rank, like the reference's jsrun resource sets (summit/run.sh:30);
# the ranks also pin themselves near their GPU when a launcher does not
# (gmt_rt_pin_rank, GMT_PIN=0 to disable); MPIRUN_BIND="" leaves it to them
bind=${MPIRUN_BIND--bind-to core}
app=$bin/mpi_daxpy_nvtx_unmanaged
[ "$um" == "um" ] && app=$bin/mpi_daxpy_nvtx_managed
np=$((nodes * ppn))
if [ "$prof" == "rocprof" ]; then
  mkdir -p profile/$tag
  export TMPDIR=${TMPDIR:-/tmp}
  $mpirun $bind -np $np rocprofv3 --marker-trace --kernel-trace --memory-copy-trace \
    --selected-regions --output-format csv -d profile/$tag/%rank% -o $tag \
    -- $app > out-${tag}.txt 2>&1
else
  $mpirun $bind -np $np $app > out-${tag}.txt 2>&1
fi
echo "wrote out-${tag}.txt"
