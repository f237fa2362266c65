#!/bin/bash
# GPU test pass on the box: the -m gpu suite (one process, per-test timeout), then smoke and a
# short bench line. Logs under gpurun_out/ (LABEL names them).
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"
L="${LABEL:-t}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > "gpurun_out/${L}_gpu_tests.log" 2>&1 || { tail -40 "gpurun_out/${L}_gpu_tests.log"; exit 1; }
tail -3 "gpurun_out/${L}_gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/${L}_smoke.log" 2>&1
tail -2 "gpurun_out/${L}_smoke.log"
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > "gpurun_out/${L}_bench.json" 2> "gpurun_out/${L}_bench.err"
  cut -c1-400 "gpurun_out/${L}_bench.json"
fi
