set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for v in pp0w4 pp1w3; do
  ICX_LIB=imagecodecs_amd/exp/libicx_$v.so ICX_FUSE420=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_foreign.py -m gpu -x -q --timeout 120 --timeout-method thread -k "plane_modes or foreign_large or golden" > gpurun_out/r03l_tests_$v.log 2>&1 || { tail -30 gpurun_out/r03l_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r03l_tests_$v.log
done
VARIANTS="pp0w4 pp1w4 pp1w3 pp0w3" REPS2=2 bash tools/gpu_back_ab.sh 2>&1 | grep -v amdgpu
