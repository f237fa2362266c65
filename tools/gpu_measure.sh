#!/bin/bash
# Round measurement on the GPU box: bench line, rocprofv3 kernel stats of the same command,
# PMC traffic of the dominant kernel. Outputs under gpurun_out/meas (copied into profiles/ after).
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/meas"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ARGS="${BENCH_ARGS:-}"
timeout -k 10 600 python3 "$R/bench.py" $ARGS > "$O/bench.json" 2> "$O/bench.err"
echo "bench: $(cut -c1-200 $O/bench.json)"
# same command without the CPU-baseline leg (its fork pool does not survive the profiler's preload)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" $ARGS --no-cpu --no-pcie > "$O/bench_rocprof.json" 2> "$O/rocprof.err"
echo "rocprof done"
timeout -k 10 1200 python3 "$R/tools/pmc_traffic.py" run --out "$O/traffic.json" --pipeline-out "$O/pipeline_traffic.json" > "$O/pmc.log" 2>&1
echo "pmc: $(tail -1 $O/pmc.log | cut -c1-300)"
