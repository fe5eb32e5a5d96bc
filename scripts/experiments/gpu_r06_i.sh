#!/bin/bash
# Round 6 (i): power and clocks under the sustained 32768^2 K = 20 pass
# (read-only rocm-smi queries while scripts/experiments/sustain.py runs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_i
mkdir -p $OUT
timeout -k 10 60 rocm-smi --showmaxpower --showpower --showclocks > $OUT/smi_idle.txt 2>&1 || true
timeout -k 10 120 python3 scripts/experiments/sustain.py 32768 30 > $OUT/sustain.txt 2>&1 &
pid=$!
for i in 1 2 3 4 5 6; do
  sleep 4
  if grep -q "sustain: start" $OUT/sustain.txt; then
    timeout -k 5 30 rocm-smi --showpower --showclocks --showtemp > $OUT/smi_busy_$i.txt 2>&1 || true
  fi
done
wait $pid || { tail -20 $OUT/sustain.txt; exit 1; }
grep -hiE "max graphics package power|power cap" $OUT/smi_idle.txt | head -4
grep -hiE "package power|sclk|fclk|junction" $OUT/smi_busy_*.txt | head -30
tail -5 $OUT/sustain.txt
echo R06I_OK
