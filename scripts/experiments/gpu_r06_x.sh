#!/bin/bash
# Round 6 (x): counters of the 32768^2 K = 20 Dirichlet pass in three launch
# shapes — one strip per workgroup (round 5), two strips stage-major (the
# default), two strips strip-major — one PMC pass and one kernel trace each
# (3 passes per run): VALU instructions, VALU-active and stall cycles, and
# the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$PWD
OUT=$R/gpurun_out/r06_x
mkdir -p $OUT
B=$R/build/bin/gmt_kernel_bench
export TMPDIR=/tmp
cd /tmp
C="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"
for v in nw1 nw2 nw2s; do
  case $v in
    nw1) nw=1; export GMT_TB_SHARED=0 GMT_TB_STRIP_MAP=1;;
    nw2) nw=2; export GMT_TB_SHARED=0 GMT_TB_STRIP_MAP=1;;
    nw2s) nw=2; export GMT_TB_SHARED=0 GMT_TB_STRIP_MAP=0;;
  esac
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$v" -o p -- "$B" --only=tb --tb-k=20 --tb-nw=$nw --tb-mask=0 --jacobi-n=32768 --iters=3 \
    > "$OUT/pmc_$v.log" 2>&1 || { echo "pmc $v failed"; tail -20 "$OUT/pmc_$v.log"; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$v" -o t -- "$B" --only=tb --tb-k=20 --tb-nw=$nw --tb-mask=0 --jacobi-n=32768 --iters=3 \
    > "$OUT/trace_$v.log" 2>&1 || { echo "trace $v failed"; tail -20 "$OUT/trace_$v.log"; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
base = "gpurun_out/r06_x"
for v in ("nw1", "nw2", "nw2s"):
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
echo R06X_OK
