#!/bin/bash
# Round 4: encoder RGB gather with dword loads -- encode GPU tests, C4 A/B against the previous build.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_encode.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c4b_tests.log 2>&1
rc=$?; echo "encode tests rc=$rc: $(tail -1 gpurun_out/r04c4b_tests.log)"; stop $rc
grep -E "^E |FAILED" gpurun_out/r04c4b_tests.log | head
[ $rc -eq 0 ] || exit $rc
for lib in; do
  ICX_LIB=imagecodecs_amd/$lib timeout -k 10 300 python3 bench.py --workload c4 --no-cpu --steps 10 --warmup 2 > gpurun_out/r04c4b_ab.json 2>gpurun_out/r04c4b_ab.err
  rc=$?; stop $rc
  echo "c4 $lib: $(python3 -c "import json;d=json.load(open('gpurun_out/r04c4b_ab.json'));print(d['value'],d['ms_per_step'],d.get('parity'))")"
done
