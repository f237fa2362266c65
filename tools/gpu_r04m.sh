#!/bin/bash
# Round 4: C2 knob sweep (lane size, path, lead, grid) with host-driven rounds.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for rep in 1 2; do
for v in "X=0" "ICX_GW=1" "ICX_GUESS_LEAD=1024" "ICX_BIG_WG=0 ICX_SUB_BYTES=1536" "ICX_SUB_BYTES=1024" "ICX_EGRID=4096" "ICX_PIPES=1"; do
  env $v timeout -k 10 200 python3 bench.py --workload c2 --no-cpu --no-pcie --steps 10 --warmup 2 > gpurun_out/r04m.json 2>/dev/null
  rc=$?; stop $rc
  echo "c2 [$v]: $(python3 -c "import json;d=json.load(open('gpurun_out/r04m.json'));print(d['value'],d['ms_per_step'],d['entropy_paths'])" 2>&1)"
done
done
