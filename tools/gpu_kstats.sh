#!/bin/bash
# Kernels-alone comparison of library builds on one GPU box: for each library in LIBS (paths under
# imagecodecs_amd/), one rocprofv3 --kernel-trace --stats pass of a short bench on ONE pipeline
# (ICX_PIPES=1, so each kernel runs alone) and a per-kernel summary. Optional PROBE=1 first runs
# tools/probe/valu_issue (the VALU issue-rate calibration) plainly and under one --pmc pass.
#   LABEL=r06a LIBS="lib/libicx.so xlib/libicx_nostore.so" BENCH_ARGS="--images 256" tools/gpu_kstats.sh
# Output: gpurun_out/<LABEL>_<lib>/ (trace), gpurun_out/<LABEL>_kstats.txt (summaries).
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd /tmp && export TMPDIR=/tmp
L="${LABEL:-ks}"
mkdir -p "$R/gpurun_out"
OUT="$R/gpurun_out/${L}_kstats.txt"; : > "$OUT"
if [ -n "${PROBE:-}" ]; then
  timeout -k 10 120 "$R/tools/probe/valu_issue" ${PROBE_ITERS:-20000} > "$R/gpurun_out/${L}_valu_issue.jsonl" 2>&1
  rc=$?; echo "valu_issue rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/${L}_valu_issue.jsonl"; exit $rc; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/${L}_valu_pmc" -o run -- "$R/tools/probe/valu_issue" ${PROBE_ITERS:-20000} \
    > "$R/gpurun_out/${L}_valu_pmc.log" 2>&1
  rc=$?; echo "valu_issue pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/${L}_valu_pmc.log"; exit $rc; }
fi
for lib in ${LIBS:-lib/libicx.so}; do
  tag=$(basename "$lib" .so)
  O="$R/gpurun_out/${L}_${tag}"; mkdir -p "$O"
  ICX_PIPES="${PIPES:-1}" ICX_LIB="$R/imagecodecs_amd/$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$O/trace" -o run -- python3 "$R/bench.py" --steps ${STEPS:-2} --warmup 1 --no-cpu --no-pcie ${BENCH_ARGS:-} \
    > "$O/bench.json" 2> "$O/err.log"
  rc=$?; echo "$tag rc=$rc $(tail -c 300 "$O/bench.json")"
  case $rc in 0|1) ;; *) tail -20 "$O/err.log"; exit $rc;; esac  # (1: a timing build's parity check may fail)
  python3 - "$O" "$tag" >> "$OUT" <<'PY'
import csv, glob, sys
O, tag = sys.argv[1], sys.argv[2]
f = glob.glob(f"{O}/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
print(f"== {tag}")
for r in rows[:14]:
    name = r["Name"].split("(")[0].replace("icx::", "").replace("void ", "")
    print(f'{name:34s} calls {int(r["Calls"]):4d} avg {float(r["AverageNs"])/1e6:8.3f} ms  total {float(r["TotalDurationNs"])/1e6:8.2f}')
PY
done
cat "$OUT"
