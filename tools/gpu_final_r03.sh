#!/bin/bash
# Round-3 end measurement on one box: the whole GPU suite, smoke, C3 bench at the driver's
# settings with rocprofv3 stats and PMC traffic (tools/gpu_measure.sh), C5 batch vs per-image.
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r03z}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${TAG:-r03z}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG:-r03z}_gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r03z}_smoke.log 2>&1
tail -1 gpurun_out/${TAG:-r03z}_smoke.log
BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_measure.sh
cd "$R"
for f in batch single; do
  x=""; [ $f = single ] && x="--png-single"
  timeout -k 10 300 python3 bench.py --workload c5 --steps 5 --warmup 1 $x > gpurun_out/${TAG:-r03z}_c5_$f.json
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], d['parity'])" gpurun_out/${TAG:-r03z}_c5_$f.json $f
done
