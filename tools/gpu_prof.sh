#!/bin/bash
# Per-kernel timing on the GPU box: rocprofv3 kernel stats of a short C3 bench with PIPES
# pipelines (1: kernels alone, 2: the default overlap). LABEL names the output dir; ICX_LIB
# (optional) selects an experiment build. Summaries under gpurun_out/prof_<LABEL>/.
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd /tmp && export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu --no-pcie}"
P="${PIPES:-1}"
O="$R/gpurun_out/prof_${LABEL:-p$P}"; mkdir -p "$O"
ICX_PIPES=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o run -- python3 "$R/bench.py" $ARGS > "$O/bench.json" 2> "$O/err.log"
python3 - "$O" <<'PY'
import csv, glob, sys
O = sys.argv[1]
f = glob.glob(f"{O}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
with open(f"{O}/summary.txt", "w") as out:
    for r in rows[:14]:
        name = r["Name"].split("(")[0].replace("icx::", "").replace("void ", "")
        line = f'{name:34s} calls {int(r["Calls"]):4d} avg {float(r["AverageNs"])/1e6:8.3f} ms'
        print(line); out.write(line + "\n")
PY
echo "--- ${LABEL:-p$P}: $(cut -c1-170 $O/bench.json)"
