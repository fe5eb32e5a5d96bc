#!/bin/bash
# Round 6 (z): counters of the shared hand-off group against two stage-major
# strips at 32768^2 with halo sides (mask 15, where their rates tie): where
# do the group's 6% fewer level updates go?
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$PWD
OUT=$R/gpurun_out/r06_z
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
export TMPDIR=/tmp
cd /tmp
C="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"
for v in sh nw2; do
  case $v in
    sh) nw=0; export GMT_TB_SHARED=1;;
    nw2) nw=2; export GMT_TB_SHARED=0;;
  esac
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$v" -o p -- "$B" --only=tb --tb-k=20 --tb-nw=$nw --tb-mask=15 --jacobi-n=32768 --iters=3 \
    > "$OUT/pmc_$v.log" 2>&1 || { echo "pmc $v failed"; tail -20 "$OUT/pmc_$v.log"; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$v" -o t -- "$B" --only=tb --tb-k=20 --tb-nw=$nw --tb-mask=15 --jacobi-n=32768 --iters=3 \
    > "$OUT/trace_$v.log" 2>&1 || { echo "trace $v failed"; tail -20 "$OUT/trace_$v.log"; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
base = "gpurun_out/r06_z"
for v in ("sh", "nw2"):
    cnt = collections.defaultdict(list)
    for f in glob.glob(f"{base}/pmc_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "jacobi5tb_kernel<20" in r.get("Kernel_Name", ""):
                cnt[(r.get("Dispatch_Id"), r["Counter_Name"])].append(float(r["Counter_Value"]))
    per = collections.defaultdict(list)
    for (d, n), vals in cnt.items():
        per[n].append(sum(vals))
    durs = []
    for f in glob.glob(f"{base}/trace_{v}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "jacobi5tb_kernel<20" in r.get("Kernel_Name", ""):
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    m = {n: sum(x) / len(x) for n, x in per.items()}
    ms = sorted(durs)[len(durs) // 2] if durs else 0
    clk = m.get("GRBM_GUI_ACTIVE", 0) / 8 / (ms * 1e-3) / 1e6 if ms else 0
    print(v, "passes", len(per.get("SQ_WAVES", [])), "ms", round(ms, 3), "clock_MHz", round(clk),
          {k: f"{x:.4g}" for k, x in sorted(m.items())})
PY
echo R06Z_OK
