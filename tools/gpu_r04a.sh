#!/bin/bash
# Round 4, first box: whole-pipeline PMC traffic of a C3 step (every kernel's FETCH/WRITE, per
# image) and the kernel-trace stats of the same bench command.
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/${TAG:-r04a}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 "$R/tools/pmc_traffic.py" run --images ${PMC_IMAGES:-128} --out "$O/traffic.json" \
  --pipeline-out "$O/pipeline_traffic.json" > "$O/pmc.log" 2>&1
echo "pmc: $(tail -1 $O/pmc.log | cut -c1-400)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu --no-pcie > "$O/bench_rocprof.json" 2> "$O/rocprof.err"
echo "bench(rocprof): $(cut -c1-200 $O/bench_rocprof.json)"
