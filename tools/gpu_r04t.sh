#!/bin/bash
# Round 4: back half non-temporal (ICX_NT_BACK=1 experiment build) A/B on C3 and C2.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for wl in c3; do
for lib in lib/libicx.so exp/libicx_nt1.so exp/libicx_nt2.so lib/libicx.so exp/libicx_nt1.so exp/libicx_nt2.so; do
  ICX_LIB=imagecodecs_amd/$lib timeout -k 10 300 python3 bench.py --workload $wl --no-cpu --no-pcie --steps 20 --warmup 5 > gpurun_out/r04t_ab.json 2>gpurun_out/r04t_ab.err
  rc=$?; stop $rc
  echo "$wl $lib: $(python3 -c "import json;d=json.load(open('gpurun_out/r04t_ab.json'));print(d['value'],d['ms_per_step'],d['entropy_paths'],d.get('parity'))")"
done
done
