#!/bin/bash
# Round 4: GPU suite, entropy-round overhead A/B, and k_gw_lane experiment builds (kernel stats).
# A failed test does not stop the measurements; a crash, abort or time limit stops everything.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04d_tests.log)"; stop $rc
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r04d_tests.log | tail -15
grep -E "4096\^2|x 512\^2|GPU IDAT" gpurun_out/r04d_tests.log | head -20
for e in "ICX_ROUNDS=1" "" "ICX_ROUNDS=1" ""; do
  env $e timeout -k 10 200 python3 bench.py --no-cpu --no-pcie --steps 10 --warmup 2 > gpurun_out/r04d_ab.json 2>/dev/null
  rc=$?; stop $rc
  echo "c3 ${e:-default}: $(python3 -c "import json;d=json.load(open('gpurun_out/r04d_ab.json'));print(d['value'],d['ms_per_step'],d['entropy_paths'])")"
done
VARS="ICX_LIB=imagecodecs_amd/lib/libicx.so ICX_LIB=imagecodecs_amd/exp/libicx_gw8.so ICX_LIB=imagecodecs_amd/exp/libicx_gw8w6.so" PMC="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" bash tools/gpu_cmp.sh 2>&1 | grep -E "==|gw_lane|idct420y|SQ k_gw_lane"
