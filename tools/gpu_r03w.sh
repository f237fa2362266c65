# Decode parity of a variant library (ICX_LIB=$LIBV) then kernel times: HEAD~ copy, tree, variant.
set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
ICX_LIB="$R/$LIBV" timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_foreign.py tests/test_gpu_fallback.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03w_tests.log 2>&1 || { tail -40 gpurun_out/r03w_tests.log; exit 1; }
tail -1 gpurun_out/r03w_tests.log
MORE="v=ICX_LIB=$LIBV" bash tools/gpu_r03v.sh
