#!/bin/bash
# Tuning aid (GPU box): the GPU test suite, then one bench line per "WORKLOAD[:VAR=VAL[,VAR=VAL]]"
# entry of ENVAB (e.g. "c2 c2:ICX_SUB_BYTES=1024 c3:ICX_GUESS_LEAD=0"), each with only that
# entry's environment overrides.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"
mkdir -p gpurun_out
if [ -z "$ENVAB_NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/envab_tests.log 2>&1 || { tail -30 gpurun_out/envab_tests.log; exit 1; }
  tail -1 gpurun_out/envab_tests.log
fi
for e in $ENVAB; do
  w=${e%%:*}; vars=""; [ "$e" != "$w" ] && vars=${e#*:}
  env ${vars//,/ } timeout -k 10 200 python bench.py --workload $w --no-cpu --no-pcie --steps ${STEPS:-10} > gpurun_out/envab.json 2>/dev/null || exit 1
  echo "$e $(python -c "import json;d=json.load(open('gpurun_out/envab.json'));print(d['value'],d['ms_per_step'])")"
done
