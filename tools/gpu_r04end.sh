#!/bin/bash
# Round 4: last check at the final code -- the whole GPU suite and smoke.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04end_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04end_gpu_tests.log)"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04end_smoke.log 2>&1
echo "smoke rc=$?: $(tail -1 gpurun_out/r04end_smoke.log)"
