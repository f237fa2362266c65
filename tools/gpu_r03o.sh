set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_foreign.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03o_tests.log 2>&1 || { tail -40 gpurun_out/r03o_tests.log; exit 1; }
tail -1 gpurun_out/r03o_tests.log
echo "== new"; timeout -k 10 300 python3 tools/seq_time.py 512 1024 2048 4096 2>&1 | grep -v amdgpu
echo "== old"; ICX_LIB=imagecodecs_amd/exp/libicx_old.so timeout -k 10 300 python3 tools/seq_time.py 512 1024 2048 2>&1 | grep -v amdgpu
