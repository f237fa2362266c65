#!/bin/bash
# Kernel-level comparison of decode variants on one box: for each entry of VARS (env settings,
# e.g. "ICX_GW=1 ICX_GW=0"), rocprofv3 kernel stats of a short C3 bench with one pipeline (kernels
# alone) and one SQ counter pass. Summaries under gpurun_out/cmp_<var>/.
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for kv in ${VARS:-ICX_GW=1}; do
  O="$R/gpurun_out/cmp_${kv//[=\/]/_}"; mkdir -p "$O"
  case "$kv" in ICX_LIB=/*) ;; ICX_LIB=*) kv="ICX_LIB=$R/${kv#ICX_LIB=}" ;; esac  # (runs from /tmp)
  export $kv
  ICX_PIPES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --no-pcie > "$O/bench.json" 2> "$O/err.log"
  ICX_PIPES=1 timeout -s KILL 180 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY} --output-format csv -d "$O/sq" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-pcie --images ${SQ_IMAGES:-128} > "$O/sq.log" 2>&1
  unset ${kv%%=*}
  python3 - "$O" "$kv" <<'PY'
import csv, glob, sys, collections
O, kv = sys.argv[1], sys.argv[2]
f = glob.glob(f"{O}/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
out = open(f"{O}/summary.txt", "w")
def p(x):
    print(x); out.write(x + "\n")
p(f"== {kv}")
for r in rows[:16]:
    name = r["Name"].split("(")[0].replace("icx::", "").replace("void ", "")
    p(f'{name:34s} calls {int(r["Calls"]):4d} avg {float(r["AverageNs"])/1e6:8.3f} ms  total {float(r["TotalDurationNs"])/1e6:8.2f}')
agg = collections.defaultdict(float)
for g in glob.glob(f"{O}/sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(g)):
        agg[(r["Kernel_Name"].split("(")[0].replace("icx::", "").replace("void ", ""), r["Counter_Name"])] += float(r["Counter_Value"])
ks = sorted({k for k, _ in agg}, key=lambda k: -agg.get((k, "SQ_WAVE_CYCLES"), 0))[:8]
G = lambda k, c: agg.get((k, c), 0.0)
extra = sorted({c for _, c in agg} - {"SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"})
for k in ks if extra else []:  # counters beyond the default set: per wave, and per wave-cycle
    w = max(1, G(k, "SQ_WAVES")); wc = max(1, G(k, "SQ_WAVE_CYCLES"))
    p(f"PMC {k:30s} " + " ".join(f"{c} {G(k, c)/w:.0f}/w ({100*G(k, c)/wc:.1f}%cyc)" for c in extra))
for k in ks:
    w = max(1, G(k, "SQ_WAVES")); wc = max(1, G(k, "SQ_WAVE_CYCLES"))
    p(f"SQ {k:30s} waves {w:8.0f} VALU/w {G(k,'SQ_INSTS_VALU')/w:9.0f} SALU/w {G(k,'SQ_INSTS_SALU')/w:8.0f} LDS/w {G(k,'SQ_INSTS_LDS')/w:7.0f} actVALU {100*G(k,'SQ_ACTIVE_INST_VALU')/wc:5.1f}% act {100*G(k,'SQ_ACTIVE_INST_ANY')/wc:5.1f}% waitinst {100*G(k,'SQ_WAIT_INST_ANY')/wc:5.1f}% cyc/w {wc/w:10.0f}")
PY
done
