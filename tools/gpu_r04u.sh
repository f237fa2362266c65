#!/bin/bash
# Round 4: C3 longest-lane sweep (ICX_SUB_MAX).
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for pass in 1 2; do
for lead in default 3072 2112 1600; do
  if [ $lead = default ]; then unset ICX_SUB_MAX; else export ICX_SUB_MAX=$lead; fi
  timeout -k 10 300 python3 bench.py --workload c3 --no-cpu --no-pcie --steps 20 --warmup 5 > gpurun_out/r04u_ab.json 2>gpurun_out/r04u_ab.err
  rc=$?; stop $rc
  echo "c3 sub_max=$lead: $(python3 -c "import json;d=json.load(open('gpurun_out/r04u_ab.json'));print(d['value'],d['ms_per_step'],d['entropy_paths'])")"
done
done
