#!/bin/bash
# Round 4: PNG (hashed LZ77 candidate) and fallback tests, C5 bench, then tools/gpu_r04c.sh (C2
# traces for both entropy paths, C3 with staggered pipelines). Stops at a crash / time limit.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_png.py tests/test_gpu_fallback.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04e_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04e_tests.log)"; stop $rc
grep -E "^FAILED|4096\^2|x 512\^2|GPU IDAT" gpurun_out/r04e_tests.log | head -20
timeout -k 10 300 python3 bench.py --workload c5 --steps 5 --warmup 1 > gpurun_out/r04e_c5.json 2>/dev/null
rc=$?; stop $rc
echo "c5: $(python3 -c "import json;d=json.load(open('gpurun_out/r04e_c5.json'));print(d['value'],d['ms_per_step'],d['config']['png_bytes_per_pixel'],d['parity'])")"
bash tools/gpu_r04c.sh
