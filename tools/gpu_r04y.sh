#!/bin/bash
# Round 4: the whole GPU suite with the one-pass unstuff (ICX_USTF1=1, v3).
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
ICX_USTF1=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04y_tests.log 2>&1
rc=$?; echo "suite (one-pass) rc=$rc: $(tail -1 gpurun_out/r04y_tests.log)"
grep -E "^E |FAILED" gpurun_out/r04y_tests.log | head -20
exit $rc
