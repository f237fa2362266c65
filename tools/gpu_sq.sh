#!/bin/bash
# SQ counter pass (one --pmc run of 8 SQ counters, no tracing domains) over a short decode bench.
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/sq"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY --output-format csv -d "$O/a" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --images ${SQ_IMAGES:-128} ${SQ_ARGS:-} > "$O/a.log" 2>&1
python3 "$R/tools/sq_summary.py" "$O/a" | tee "$O/summary.txt"
