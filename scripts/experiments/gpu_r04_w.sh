#!/bin/bash
# Round 4 (w): the driver-config bench under a kernel trace: how long is the
# one timed 20-sweep pass on the GPU against the host-timed ms_per_step x 20?
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
R=$PWD
OUT=$R/${OUT:-gpurun_out/r04_w}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --skip-extras --skip-check > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
tail -1 $OUT/b.json | cut -c1-300
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/tr/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
tb = [r for r in rows if "jacobi5tb_kernel" in r["Kernel_Name"]]
for r in tb[-6:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(r["Kernel_Name"].split("(")[0][-40:], r["Grid_Size_X"], f"{(e - s) / 1e6:.4f} ms", s)
PY
