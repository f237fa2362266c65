#!/bin/bash
# Round 4: EXR inflate with the chunked bit reader and 4-byte match copies -- EXR GPU tests, EXR bench.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_exr.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04z2_exr_tests.log 2>&1
rc=$?; echo "exr tests rc=$rc: $(tail -1 gpurun_out/r04z2_exr_tests.log)"; stop $rc
grep -E "^E |FAILED" gpurun_out/r04z2_exr_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for lib in exp/libicx_exrring.so lib/libicx.so exp/libicx_exrring.so lib/libicx.so; do
  ICX_LIB=imagecodecs_amd/$lib timeout -k 10 400 python3 bench.py --workload exr --steps 5 --warmup 2 --no-cpu > gpurun_out/r04z2_ab.json 2> gpurun_out/r04z2_ab.err
  rc=$?; stop $rc
  echo "exr $lib: $(python3 -c "import json;d=json.load(open('gpurun_out/r04z2_ab.json'));print(d['value'],d['ms_per_step'],d.get('parity'))")"
done
timeout -k 10 400 python3 bench.py --workload exr --steps 5 --warmup 2 > gpurun_out/r04z2_bench_exr.json 2> gpurun_out/r04z2_bench_exr.err
rc=$?; echo "bench exr rc=$rc: $(cut -c1-200 gpurun_out/r04z2_bench_exr.json)"; stop $rc
