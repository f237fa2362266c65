#!/bin/bash
# A/B of environment settings on one box: for each entry of AB (e.g. "ICX_GW=1 ICX_GW=0"), a C3
# bench line with that variable set (REPS rounds, interleaved). Lines under gpurun_out/ab_*.json.
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
ARGS="${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu --no-pcie}"
for rep in $(seq 1 ${REPS:-1}); do
  for kv in ${AB:-ICX_GW=1}; do
    env $kv timeout -k 10 300 python3 bench.py $ARGS > "gpurun_out/ab_${kv//[=\/]/_}_$rep.json"
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], {k:round(v,2) for k,v in d['roofline']['stage_ms'].items()}, d['entropy_paths'], d['parity'])" "gpurun_out/ab_${kv//[=\/]/_}_$rep.json" "$kv"
  done
done
