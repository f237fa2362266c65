#!/bin/bash
# C2 entropy-path sweep on one box: each "ENV=..." setting of SETS (';'-separated) runs one C2
# bench (steps 10, warmup 3); prints GP/s per setting.
#   SETS="ICX_GW=0;ICX_GW=1 ICX_SUB_BYTES=1024" tools/gpu_c2sweep.sh
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R" || exit 1
mkdir -p gpurun_out
IFS=';' read -ra SS <<< "${SETS:-ICX_GW=0}"
k=0
for s in "${SS[@]}"; do
  k=$((k + 1))
  env $s timeout -k 10 300 python3 bench.py --workload ${WL:-c2} --steps ${STEPS:-10} --warmup 3 --no-cpu --no-pcie \
    > gpurun_out/c2s$k.json 2> gpurun_out/c2s$k.err || { echo "$s failed"; tail -5 gpurun_out/c2s$k.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c2s$k.json').read().splitlines()[-1]); print('$s', round(d['value']/1000, 2), d['ms_per_step'], d.get('parity'))"
done
