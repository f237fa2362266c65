#!/bin/bash
# Round 4: EXR bench kernel split (rocprofv3 kernel trace + stats).
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/r04e2"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --workload exr --steps 3 --warmup 1 --no-cpu > "$O/bench.json" 2> "$O/err.log"
echo "rc=$? $(cut -c1-120 $O/bench.json)"
