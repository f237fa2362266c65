#!/bin/bash
# Round 4: k_idct420c compiled for 4 waves per SIMD (ICX_IDCT_C_MINW=4, 128 VGPRs + 24 B scratch) A/B on C3.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for lib in lib/libicx.so exp/libicx_ic4.so lib/libicx.so exp/libicx_ic4.so; do
  ICX_LIB=imagecodecs_amd/$lib timeout -k 10 300 python3 bench.py --workload c3 --no-cpu --no-pcie --steps 20 --warmup 5 > gpurun_out/r04ic_ab.json 2>gpurun_out/r04ic_ab.err
  rc=$?; stop $rc
  echo "c3 $lib: $(python3 -c "import json;d=json.load(open('gpurun_out/r04ic_ab.json'));print(d['value'],d['ms_per_step'],d['entropy_paths'])")"
done
