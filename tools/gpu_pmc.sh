#!/bin/bash
# Per-kernel HBM traffic (FETCH_SIZE / WRITE_SIZE, separate --pmc passes) of a short C3 decode,
# plus an SQ instruction/wait pass. ICX_LIB (optional) selects an experiment build; LABEL names
# the output dir gpurun_out/pmc_<LABEL>/ (summary.txt).
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/pmc_${LABEL:-x}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-pcie --images ${PMC_IMAGES:-128}"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- $B > "$O/fetch.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- $B > "$O/write.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM --output-format csv -d "$O/sq" -o run -- $B > "$O/sq.log" 2>&1
python3 - "$O" <<'PY' | tee "$O/summary.txt"
import csv, glob, sys, collections
O = sys.argv[1]
agg = collections.defaultdict(float)
for sub in ("fetch", "write", "sq"):
    for f in glob.glob(f"{O}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("icx::", "").replace("void ", "")
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
ks = sorted({k for k, _ in agg}, key=lambda k: -agg.get((k, "SQ_WAVE_CYCLES"), 0))
g = lambda k, c: agg.get((k, c), 0.0)
print(f"{'kernel':24s} {'fetchMB(x2)':>11s} {'writeMB':>9s} {'VALU/w':>8s} {'LDS/w':>7s} {'VMEM/w':>7s} {'wait%':>6s} {'issue%':>6s} {'actVALU%':>8s}")
for k in ks:
    wc = g(k, "SQ_WAVE_CYCLES"); w = max(1, g(k, "SQ_WAVES"))
    if wc <= 0: continue
    print(f"{k:24s} {2*g(k,'FETCH_SIZE')/1024:11.1f} {g(k,'WRITE_SIZE')/1024:9.1f} {g(k,'SQ_INSTS_VALU')/w:8.0f} {g(k,'SQ_INSTS_LDS')/w:7.0f} {g(k,'SQ_INSTS_VMEM')/w:7.0f} "
          f"{100*g(k,'SQ_WAIT_ANY')/wc:6.1f} {100*g(k,'SQ_WAIT_INST_ANY')/wc:6.1f} {100*g(k,'SQ_ACTIVE_INST_VALU')/wc:8.1f}")
PY
