#!/bin/bash
# Round 4: encode device batch at an odd file stride.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_encode.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04w.log 2>&1
rc=$?; echo "rc=$rc: $(tail -1 gpurun_out/r04w.log)"; grep -E "^E |FAILED" gpurun_out/r04w.log | head
