#!/bin/bash
# Round 4: one-pass unstuff (ICX_USTF1=1) -- decode tests, then C3/C2 A/B, then the whole GPU suite with it.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
ICX_USTF1=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decode.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04x_decode.log 2>&1
rc=$?; echo "decode tests (one-pass) rc=$rc: $(tail -1 gpurun_out/r04x_decode.log)"; stop $rc
grep -E "^E |FAILED" gpurun_out/r04x_decode.log | head -20
[ $rc -eq 0 ] || exit $rc
for wl in c3 c2; do
for one in 0 1 0 1; do
  ICX_USTF1=$one timeout -k 10 300 python3 bench.py --workload $wl --no-cpu --no-pcie --steps 20 --warmup 5 > gpurun_out/r04x_ab.json 2>gpurun_out/r04x_ab.err
  rc=$?; stop $rc
  echo "$wl ICX_USTF1=$one: $(python3 -c "import json;d=json.load(open('gpurun_out/r04x_ab.json'));print(d['value'],d['ms_per_step'],d['entropy_paths'],d.get('parity'))")"
done
done
[ -n "$FULL" ] && ICX_USTF1=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04x_tests.log 2>&1
rc=$?; echo "suite (one-pass) rc=$rc: $(tail -1 gpurun_out/r04x_tests.log)"; stop $rc
grep -E "^E |FAILED" gpurun_out/r04x_tests.log | head -20
