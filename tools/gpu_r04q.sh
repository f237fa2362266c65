#!/bin/bash
# Round 4: C3 kernels alone (one pipeline), full list, current build.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/r04q"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
ICX_PIPES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu --no-pcie > "$O/bench.json" 2> "$O/err.log"
echo "rc=$? $(cut -c1-120 $O/bench.json)"
