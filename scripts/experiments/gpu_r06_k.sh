#!/bin/bash
# Round 6 (k): power, clocks and temperature under sustained K = 20 passes of
# 32768^2 and of 8192^2 (read-only rocm-smi queries while
# scripts/experiments/sustain.py runs): is the ~1.9 GHz of the headline a
# power cap?
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r06_k
mkdir -p $OUT
timeout -k 10 60 rocm-smi --showmaxpower --showpower --showclocks --showtemp > $OUT/smi_idle.txt 2>&1 || true
timeout -k 10 60 rocm-smi --showpowerlimit --showperflevel --showvoltage > $OUT/smi_limits.txt 2>&1 || true
for n in 32768 8192; do
  timeout -k 10 120 python3 scripts/experiments/sustain.py $n 30 > $OUT/sustain_$n.txt 2>&1 &
  pid=$!
  for i in 1 2 3 4 5 6; do
    sleep 4
    if grep -q "sustain: start" $OUT/sustain_$n.txt; then
      timeout -k 5 30 rocm-smi --showpower --showclocks --showtemp > $OUT/smi_busy_${n}_$i.txt 2>&1 || true
    fi
  done
  wait $pid || { tail -20 $OUT/sustain_$n.txt; exit 1; }
  tail -3 $OUT/sustain_$n.txt
done
cat $OUT/smi_idle.txt $OUT/smi_limits.txt | grep -vE "^=+|^$" | head -40
for f in $OUT/smi_busy_*; do echo "== $f"; grep -iE "power|sclk|fclk|mclk|temp" $f | head -12; done
echo R06K_OK
