#!/bin/bash
# job.sh — the reference's job matrix (summit/job.lsf, jlse/job.pbs) on one
# MI355X node: unmanaged runs at 8/4/2 ranks (one per GPU), with and without
# rocprofv3, then the averages.  Each step has its own time limit.  Ranks are
# bound one core each (run.sh: mpirun -bind-to core, MPIRUN_BIND to change).
set -u
cd "$(dirname "$0")/.."
mkdir -p runs && cd runs
for ppn in ${PPN_LIST:-8 4 2}; do
  timeout -k 10 300 ../scripts/run.sh noum none 1 $ppn || exit $?
  timeout -k 10 600 ../scripts/run.sh noum rocprof 1 $ppn || exit $?
done
../scripts/avg.sh gather
../scripts/avg.sh kernel
