#!/bin/bash
# Round 6 (e): rank pinning with SMT groups checked (a sibling list wider
# than 4 CPUs is not a core), pinned before MPI_Init, against unpinned and
# mpirun -bind-to core; the box's CPU topology as sysfs reports it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_e
mkdir -p $OUT
{
  for c in 0 1 2 31 32 128; do echo "cpu$c siblings: $(cat /sys/devices/system/cpu/cpu$c/topology/thread_siblings_list 2>/dev/null) core_id $(cat /sys/devices/system/cpu/cpu$c/topology/core_id 2>/dev/null) pkg $(cat /sys/devices/system/cpu/cpu$c/topology/physical_package_id 2>/dev/null)"; done
  for n in /sys/devices/system/node/node*; do echo "$(basename $n): $(cat $n/cpulist)"; done
  python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('gpu0 pci', getattr(p,'pci_domain_id',None), getattr(p,'pci_bus_id',None), getattr(p,'pci_device_id',None))"
  for d in /sys/bus/pci/devices/*/numa_node; do v=$(cat $d); [ -e "$(dirname $d)/drm" ] && echo "$(dirname $d) numa $v"; done
} > $OUT/topology.txt 2>&1
cat $OUT/topology.txt
M=/opt/conda/bin/mpirun
: > $OUT/pin_modes.txt
for rep in 1 2 3 4 5; do
  for mode in pin none bind; do
    env=""; b=""
    case $mode in none) env="GMT_PIN=0";; bind) env="GMT_PIN=0"; b="-bind-to core";; esac
    env $env timeout -k 10 120 $M $b -np 2 build/bin/mpi_halo_bench 8388608 8388608 30 --transport=mpi-host > $OUT/halo_${mode}_$rep.txt 2>&1 || { tail $OUT/halo_${mode}_$rep.txt; exit 1; }
    env $env timeout -k 10 120 $M $b -np 2 build/bin/mpi_stencil2d_sycl 1024 1 > $OUT/sycl_${mode}_$rep.txt 2>&1 || { tail $OUT/sycl_${mode}_$rep.txt; exit 1; }
    echo "rep $rep $mode: $(grep 'pinned cpu' $OUT/halo_${mode}_$rep.txt) | $(grep -E '^ *8388608' $OUT/halo_${mode}_$rep.txt | head -1) | sycl $(grep 'exchange time' $OUT/sycl_${mode}_$rep.txt | tr '\n' ' ')" | tee -a $OUT/pin_modes.txt
  done
done
echo R06E_OK
