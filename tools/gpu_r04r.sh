#!/bin/bash
# Round 4: device-resident EXR read -- EXR GPU tests, the exr bench workload.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_exr.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04r_exr_tests.log 2>&1
rc=$?; echo "exr tests rc=$rc: $(tail -1 gpurun_out/r04r_exr_tests.log)"; stop $rc
grep -E "^FAILED|^ERROR" gpurun_out/r04r_exr_tests.log | head
timeout -k 10 600 python3 bench.py --workload exr --steps 5 --warmup 2 > gpurun_out/r04r_bench_exr.json 2> gpurun_out/r04r_bench_exr.err
rc=$?; echo "exr bench rc=$rc: $(cut -c1-400 gpurun_out/r04r_bench_exr.json)"; stop $rc
tail -3 gpurun_out/r04r_bench_exr.err
