#!/bin/bash
# Round 4: C5 kernel trace (PNG encode with segment seams and merged blocks).
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/r04p"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --workload c5 --steps 5 --warmup 1 --no-cpu --no-pcie > "$O/c5.json" 2> "$O/c5.err"
echo "rc=$? $(cut -c1-200 $O/c5.json)"
