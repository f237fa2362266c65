#!/bin/bash
# Round 4: C4 encode bench and its kernel split (rocprofv3 kernel trace + stats).
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/r04c4"; mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 bench.py --workload c4 --steps 10 --warmup 2 --no-cpu > "$O/bench.json" 2> "$O/bench.err"
echo "bench rc=$? $(cut -c1-200 $O/bench.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --workload c4 --steps 5 --warmup 1 --no-cpu > "$O/bench_prof.json" 2> "$O/err.log"
echo "rc=$?"
