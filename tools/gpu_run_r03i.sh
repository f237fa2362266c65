set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
LABEL=r03i PYTEST_ARGS="tests/test_gpu_foreign.py tests/test_gpu_decode.py tests/test_gpu_exr.py" NO_BENCH=1 bash tools/gpu_tests.sh
BENCH_ARGS="--workload c2048 --steps 10 --warmup 2 --no-cpu --no-pcie" AB="ICX_GW=1 ICX_GW=0" bash tools/gpu_ab.sh > gpurun_out/ab_c2048.txt 2>&1
BENCH_ARGS="--workload c2 --steps 10 --warmup 2 --no-cpu --no-pcie" AB="ICX_GW=0" bash tools/gpu_ab.sh > gpurun_out/ab_c2.txt 2>&1
grep -v amdgpu gpurun_out/ab_c2048.txt gpurun_out/ab_c2.txt | cut -c1-200
timeout -k 10 300 python3 tools/exr_time.py 2048 2>&1 | grep -v amdgpu
