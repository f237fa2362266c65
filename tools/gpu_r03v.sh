# Per-kernel times (rocprofv3, kernels alone) of HEAD's library, the working tree and variants.
set -e
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
VARIANTS="head=ICX_LIB=imagecodecs_amd/exp/libicx_head.so new=ICX_X=0 ${MORE:-}" bash tools/gpu_kstats.sh 2>&1 | grep -v amdgpu | grep -E "==|convert|idct|gw_lane"
VARIANTS="head2=ICX_LIB=imagecodecs_amd/exp/libicx_head.so ${MORE:-} new2=ICX_X=0" bash tools/gpu_kstats.sh 2>&1 | grep -v amdgpu | grep -E "==|convert|idct|gw_lane"
