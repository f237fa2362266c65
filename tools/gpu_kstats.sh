#!/bin/bash
# Kernel stats (rocprofv3, one pipeline: kernels alone) of a short C3 bench per variant.
# VARIANTS: label=ENV1,ENV2 ... (ICX_LIB paths relative to the repo). Summaries in gpurun_out/ks_<label>.txt
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in $VARIANTS; do
  lab=${v%%=*}; envs=${v#*=}
  O="$R/gpurun_out/ks_$lab"; mkdir -p "$O"
  E=(); IFS=',' read -ra kvs <<< "$envs"
  for kv in "${kvs[@]}"; do case "$kv" in ICX_LIB=*) kv="ICX_LIB=$R/${kv#ICX_LIB=}";; esac; E+=("$kv"); done
  env "${E[@]}" ICX_PIPES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --no-pcie ${BENCH_EXTRA:-} > "$O/bench.json" 2> "$O/err.log"
  python3 - "$O" "$lab" <<'PY'
import csv, glob, sys
O, lab = sys.argv[1], sys.argv[2]
f = glob.glob(f"{O}/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows if "records" not in r["Name"]) / 1e6
out = open(f"{O}/summary.txt", "w")
def p(x):
    print(x); out.write(x + "\n")
p(f"== {lab}  (all kernels but records: {tot/3:.2f} ms per call-set)")
for r in rows[:9]:
    name = r["Name"].split("(")[0].replace("icx::", "").replace("void ", "")
    p(f'{name:34s} calls {int(r["Calls"]):4d} avg {float(r["AverageNs"])/1e6:8.3f} ms')
PY
done
