#!/bin/bash
# Round 4: PNG segment seams (overhanging matches) -- PNG GPU tests with the size ratios, C5 bench.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_png.py -m gpu -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04i_png.log 2>&1
rc=$?; echo "png tests rc=$rc: $(tail -1 gpurun_out/r04i_png.log)"; stop $rc
grep -E "^FAILED|^ERROR|zlib-6|GPU IDAT" gpurun_out/r04i_png.log | head -30
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload c5 --no-cpu --no-pcie --steps 5 --warmup 1 > gpurun_out/r04i_c5.json 2> gpurun_out/r04i_c5.err
  rc=$?; stop $rc
  python3 -c "import json;d=json.load(open('gpurun_out/r04i_c5.json'));print('c5',d['value'],d['ms_per_step'],d.get('stage_ms'),d.get('compression'))"
done
