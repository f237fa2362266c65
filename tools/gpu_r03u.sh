# Decode parity (plane modes, foreign streams) then a C3 A/B of the working tree against HEAD's
# library (imagecodecs_amd/exp/libicx_head.so), bench and per-kernel times.
set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_foreign.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03u_tests.log 2>&1 || { tail -40 gpurun_out/r03u_tests.log; exit 1; }
tail -1 gpurun_out/r03u_tests.log
run() { local lab=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-pcie > gpurun_out/u_$lab.json; python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/u_$lab.json $lab; }
for rep in 1 2; do run head ICX_LIB=imagecodecs_amd/exp/libicx_head.so; run new ICX_X=0; done
VARIANTS="head=ICX_LIB=imagecodecs_amd/exp/libicx_head.so new=ICX_X=0" bash tools/gpu_kstats.sh 2>&1 | grep -v amdgpu | grep -E "==|convert|idct|gw_lane"
