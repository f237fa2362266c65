set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
export ICX_FUSE420=3
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_foreign.py -m gpu -x -q --timeout 120 --timeout-method thread -k "plane_modes or crafted_big or foreign_large or golden or synth_large or unaligned" > gpurun_out/r03k_tests.log 2>&1 || { tail -30 gpurun_out/r03k_tests.log; exit 1; }
tail -3 gpurun_out/r03k_tests.log
BENCH_ARGS="--steps 10 --warmup 2 --no-cpu --no-pcie" AB="ICX_FUSE420=2 ICX_FUSE420=3" bash tools/gpu_ab.sh > gpurun_out/r03k_ab.txt 2>&1
grep -v amdgpu gpurun_out/r03k_ab.txt | cut -c1-220
VARS="ICX_FUSE420=3" bash tools/gpu_cmp.sh > gpurun_out/r03k_cmp.txt 2>&1; grep -v amdgpu gpurun_out/r03k_cmp.txt | head -30
