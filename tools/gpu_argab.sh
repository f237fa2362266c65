#!/bin/bash
# A/B of bench.py argument sets on one GPU box, interleaved REPS times (box-to-box spread is larger
# than most single changes). Each entry of ARGS (';'-separated) is one bench.py argument list.
#   LABEL=r06f REPS=2 ARGS="--workload c2;--workload c2 --inflight 2" tools/gpu_argab.sh
# Leading NAME=VALUE words of an entry are environment settings for that run only
# ("ICX_GW=1 --workload c2").
# Output: gpurun_out/<LABEL>_argab.txt (one JSON line per run, tagged with its arguments).
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R" || exit 1
L="${LABEL:-argab}"; REPS="${REPS:-2}"
mkdir -p gpurun_out
OUT="gpurun_out/${L}_argab.txt"; : > "$OUT"
IFS=';' read -ra AS <<< "${ARGS:---workload c3}"
for rep in $(seq 1 "$REPS"); do
  for a in "${AS[@]}"; do
    envs=(); args=()
    for w in $a; do
      if [ ${#args[@]} -eq 0 ] && [[ "$w" =~ ^[A-Z_][A-Z0-9_]*= ]]; then envs+=("$w"); else args+=("$w"); fi
    done
    env "${envs[@]}" timeout -k 10 300 python3 bench.py --no-cpu --no-pcie ${COMMON:-} "${args[@]}" > gpurun_out/${L}_one.json 2> gpurun_out/${L}_one.err
    rc=$?
    echo "{\"args\": \"$a\", \"rep\": $rep, \"rc\": $rc, \"line\": $(tail -1 gpurun_out/${L}_one.json || echo null)}" >> "$OUT"
    python3 - "$a" gpurun_out/${L}_one.json <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    print(f"{sys.argv[1]:40s} {d['value'] / 1000:8.2f} GP/s {d['ms_per_step']:8.3f} ms/step paths {d.get('entropy_paths')} ok {d['parity']['all_status_ok']} rec {d['records']['repeats_consistent']}")
except Exception as e:
    print(sys.argv[1], "no result", e)
PY
    [ $rc -eq 0 ] || { tail -20 gpurun_out/${L}_one.err; exit $rc; }
  done
done
