#!/bin/bash
# LDS/VALU SQ counters + HBM traffic (FETCH_SIZE / WRITE_SIZE passes) for the decode kernels.
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/sq2"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --images ${SQ_IMAGES:-128}"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d "$O/lds" -o run -- $B > "$O/lds.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- $B > "$O/fetch.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- $B > "$O/write.log" 2>&1
python3 - "$O" <<'PY' | tee "$O/summary.txt"
import csv, glob, sys, collections
O = sys.argv[1]
agg = collections.defaultdict(float)
for sub in ("lds", "fetch", "write"):
    for f in glob.glob(f"{O}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("icx::", "").replace("void ", "")
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
ks = sorted({k for k, _ in agg}, key=lambda k: -agg.get((k, "SQ_WAVE_CYCLES"), 0))
g = lambda k, c: agg.get((k, c), 0.0)
print(f"{'kernel':24s} {'VALU/w':>8s} {'LDS/w':>7s} {'bankcf/LDS':>10s} {'actLDS%':>7s} {'waitLDS%':>8s} {'actVALU%':>8s} {'fetchMB':>9s} {'writeMB':>9s}")
for k in ks:
    wc = g(k, "SQ_WAVE_CYCLES"); w = max(1, g(k, "SQ_WAVES"))
    if wc <= 0: continue
    print(f"{k:24s} {g(k,'SQ_INSTS_VALU')/w:8.0f} {g(k,'SQ_INSTS_LDS')/w:7.0f} {g(k,'SQ_LDS_BANK_CONFLICT')/max(1,g(k,'SQ_INSTS_LDS')):10.2f} "
          f"{100*g(k,'SQ_ACTIVE_INST_LDS')/wc:7.1f} {100*g(k,'SQ_WAIT_INST_LDS')/wc:8.1f} {100*g(k,'SQ_ACTIVE_INST_VALU')/wc:8.1f} "
          f"{2*g(k,'FETCH_SIZE')/1024:9.1f} {g(k,'WRITE_SIZE')/1024:9.1f}")
PY
