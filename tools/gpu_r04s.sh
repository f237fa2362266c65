#!/bin/bash
# Round 4: the half-flat full-group pool test.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fallback.py -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider -k half_flat > gpurun_out/r04s.log 2>&1
rc=$?; echo "rc=$rc: $(tail -1 gpurun_out/r04s.log)"; grep -E "^E |assert" gpurun_out/r04s.log | head
