#!/bin/bash
# Round 4: more decode pipelines (experiment build with up to 4), C2 and C3.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for wl in c2 c3; do
for rep in 1 2; do
for v in "ICX_PIPES=2" "ICX_PIPES=3" "ICX_PIPES=4"; do
  ICX_LIB=imagecodecs_amd/exp/libicx_p4.so env $v timeout -k 10 200 python3 bench.py --workload $wl --no-cpu --no-pcie --steps 10 --warmup 2 > gpurun_out/r04n.json 2>/dev/null
  rc=$?; stop $rc
  echo "$wl [$v]: $(python3 -c "import json;d=json.load(open('gpurun_out/r04n.json'));print(d['value'],d['ms_per_step'],d['entropy_paths'])" 2>&1)"
done
done
done
