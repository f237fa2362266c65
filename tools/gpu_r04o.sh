#!/bin/bash
# Round 4: layout flag from k_parse (no k_layout launch) -- GPU suite, C3 and C2 A/B against the previous build.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04o_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04o_tests.log)"; stop $rc
grep -E "^FAILED|^ERROR|4096\^2" gpurun_out/r04o_tests.log | head -15
[ $rc -eq 0 ] || exit $rc
for wl in c3 c2; do
for lib in exp/libicx_prev.so lib/libicx.so exp/libicx_prev.so lib/libicx.so; do
  ICX_LIB=imagecodecs_amd/$lib timeout -k 10 300 python3 bench.py --workload $wl --no-cpu --no-pcie --steps 20 --warmup 5 > gpurun_out/r04o_ab.json 2>/dev/null
  rc=$?; stop $rc
  echo "$wl $lib: $(python3 -c "import json;d=json.load(open('gpurun_out/r04o_ab.json'));print(d['value'],d['ms_per_step'],d['entropy_paths'])")"
done
done
