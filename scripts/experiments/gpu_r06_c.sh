#!/bin/bash
# Round 6 (c): the segment planner's rule-path cost above round 5's sweep
# (which rose monotonically to its top value 1.8 at 8192^2), Dirichlet sides,
# alternating reps, same box; the kernel trace of the 8192^2 bench pattern
# (1000 sweeps = 50 passes: kernel time against wall time).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r06_c
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
: > $OUT/rates.log
for rep in $([ "${SWEEP:-1}" = 1 ] && echo 1 2); do
  for shp in "--jacobi-n=8192 --iters=200" "--jacobi-ny=8192 --jacobi-nx=16384 --iters=60" "--jacobi-ny=16384 --jacobi-nx=8192 --iters=60" "--jacobi-n=32768 --iters=20"; do
    for c in 1.8 2.1 2.4 2.8 3.3; do
      echo "== c$c $shp" >> $OUT/rates.log
      GMT_TB_RULE_COST=$c timeout -k 10 200 $B --only=tb --sustained=1 --tb-k=20 --tb-mask=0 $shp >> $OUT/rates.log 2>&1 || { tail -20 $OUT/rates.log; exit 1; }
    done
  done
done
[ "${SWEEP:-1}" = 1 ] && grep -E "^==|MLUPS" $OUT/rates.log | paste - - | awk '{print $2, $3, $4, $(NF-13), $(NF-5), $(NF-4), $(NF-3), $(NF-2)}'
cd $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace8192 -o t -- python3 $R/scripts/experiments/clock_ab.py 8192 1000 2 > $OUT/trace8192.log 2>&1 || { tail -20 $OUT/trace8192.log; exit 1; }
grep "^n " $OUT/trace8192.log
# power and clocks while the 32768^2 pass runs back to back (read-only SMI queries)
timeout -k 10 120 python3 $R/scripts/experiments/clock_ab.py 32768 20 60 > $OUT/clock_long.txt 2>&1 &
cpid=$!
sleep 12
for i in 1 2 3; do
  timeout -k 5 30 rocm-smi --showpower --showclocks --showtemp > $OUT/smi_$i.txt 2>&1 || true
  sleep 2
done
wait $cpid || { tail -20 $OUT/clock_long.txt; exit 1; }
grep -hiE "power|sclk|fclk|mclk|temp" $OUT/smi_*.txt | head -30
tail -4 $OUT/clock_long.txt
# the 8192^2 extra: bench.py's default warm-up (2000 sweeps) against round 5's 10, alternating
for rep in 1 2; do
  for w in 10 2000; do
    timeout -k 10 300 python -u $R/bench.py --gpus 1 --steps 20 --warmup 5 --small-warmup $w --skip-check > $OUT/bench_w${w}_$rep.out 2> $OUT/bench_w${w}_$rep.err || { tail -30 $OUT/bench_w${w}_$rep.err; exit 1; }
    tail -1 $OUT/bench_w${w}_$rep.out > $OUT/bench_w${w}_$rep.json
    python3 -c "
import json; d = json.load(open('$OUT/bench_w${w}_$rep.json'))
print('small warm-up $w rep $rep', d['value'], d['timed_pass_sclk_mhz'], d.get('stencil_8192_MLUPS'), d.get('stencil_8192_sclk_mhz'), d.get('stencil_8192_pass_plan'), d.get('stencil_8192_check_mismatches'))"
  done
done
# where the 2-rank (one GPU shared) pass loses against one rank: the native
# app at 32768^2, 1 rank / 2 ranks IPC serial / 2 ranks push, then the same
# under a per-rank kernel trace
M=/opt/conda/bin/mpirun
J=$R/build/bin/mpi_jacobi2d
for rep in 1 2; do
  timeout -k 10 120 $J 32768 200 --tblock --tsteps=20 --warmup=40 > $OUT/j1_$rep.txt 2>&1 || { tail $OUT/j1_$rep.txt; exit 1; }
  timeout -k 10 120 $M -np 2 $J 32768 200 --tblock --tsteps=20 --warmup=40 --transport=ipc --no-overlap > $OUT/j2ipc_$rep.txt 2>&1 || { tail $OUT/j2ipc_$rep.txt; exit 1; }
  timeout -k 10 120 $M -np 2 $J 32768 200 --tblock --tsteps=20 --warmup=40 --transport=ipc --push > $OUT/j2push_$rep.txt 2>&1 || { tail $OUT/j2push_$rep.txt; exit 1; }
  echo "rep $rep: 1 rank $(grep 'TIME step' $OUT/j1_$rep.txt) | 2 ipc $(grep 'TIME step' $OUT/j2ipc_$rep.txt) | 2 push $(grep 'TIME step' $OUT/j2push_$rep.txt)"
done
for m in ipc push; do
  o="--no-overlap"; [ $m = push ] && o="--push"
  timeout -k 10 180 $M -np 2 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_n2_$m/%rank% -o k -- $J 32768 200 --tblock --tsteps=20 --warmup=40 --transport=ipc $o > $OUT/trace_n2_$m.log 2>&1 || { tail -20 $OUT/trace_n2_$m.log; exit 1; }
  grep 'TIME step' $OUT/trace_n2_$m.log
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_n1 -o k -- $J 32768 200 --tblock --tsteps=20 --warmup=40 > $OUT/trace_n1.log 2>&1 || { tail -20 $OUT/trace_n1.log; exit 1; }
grep 'TIME step' $OUT/trace_n1.log
echo R06C_OK
