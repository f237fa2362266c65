#!/bin/bash
# Round 4: int8 coefficient cells -- GPU suite (escaped-block tests included), kernel comparison
# against the int16 build and the 6-waves build, C3 bench A/B.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04j_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04j_tests.log)"; stop $rc
grep -E "^FAILED|^ERROR|Error|error" gpurun_out/r04j_tests.log | head -15
[ $rc -eq 0 ] || exit $rc
for lib in exp/libicx_int16.so lib/libicx.so exp/libicx_gw6.so exp/libicx_int16.so lib/libicx.so exp/libicx_gw6.so; do
  ICX_LIB=imagecodecs_amd/$lib timeout -k 10 200 python3 bench.py --no-cpu --no-pcie --steps 10 --warmup 2 > gpurun_out/r04j_ab.json 2>/dev/null
  rc=$?; stop $rc
  echo "c3 $lib: $(python3 -c "import json;d=json.load(open('gpurun_out/r04j_ab.json'));print(d['value'],d['ms_per_step'],d['entropy_paths'])")"
done
VARS="ICX_LIB=imagecodecs_amd/exp/libicx_int16.so ICX_LIB=imagecodecs_amd/lib/libicx.so ICX_LIB=imagecodecs_amd/exp/libicx_gw6.so" bash tools/gpu_cmp.sh 2>&1 | grep -E "==|gw_lane|idct420|convert_stream|gw_count|SQ k_gw_lane"
