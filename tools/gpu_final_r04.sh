#!/bin/bash
# Round-4 end measurement on one box: the whole GPU suite, smoke, C3 bench at the driver's
# settings with rocprofv3 stats, PMC traffic of k_gw_lane and of the whole pipeline (every kernel
# of a 512-image step; only with PMC=1), C2 at the driver's settings, C5 batch, EXR batch, C4 encode. Stops at the first GPU fault,
# abort or time limit.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
T=${TAG:-r04z}
stop() { case $1 in 0) ;; 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; *) echo "step failed: $1";; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/${T}_gpu_tests.log)"; stop $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/${T}_smoke.log)"; stop $rc
O="$R/gpurun_out/$T"; mkdir -p "$O"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$O/bench_c3.json" 2> "$O/bench_c3.err"
rc=$?; echo "c3: $(cut -c1-160 $O/bench_c3.json)"; stop $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu --no-pcie > "$O/bench_c3_rocprof.json" 2> "$O/rocprof.err"
rc=$?; echo "rocprof rc=$rc"; stop $rc
[ -n "$PMC" ] && timeout -k 10 1200 python3 "$R/tools/pmc_traffic.py" run --out "$O/traffic.json" --pipeline-out "$O/pipeline_traffic.json" > "$O/pmc.log" 2>&1
rc=$?; [ -n "$PMC" ] && echo "pmc rc=$rc: $(tail -1 $O/pmc.log | cut -c1-200)" && stop $rc
cd "$R"
timeout -k 10 600 python3 bench.py --workload c2 --steps 20 --warmup 5 > "$O/bench_c2.json" 2> "$O/bench_c2.err"
rc=$?; echo "c2: $(cut -c1-160 $O/bench_c2.json)"; stop $rc
timeout -k 10 600 python3 bench.py --workload c5 --steps 5 --warmup 1 > "$O/bench_c5.json" 2> "$O/bench_c5.err"
rc=$?; echo "c5: $(cut -c1-160 $O/bench_c5.json)"; stop $rc
timeout -k 10 600 python3 bench.py --workload exr --steps 5 --warmup 2 > "$O/bench_exr.json" 2> "$O/bench_exr.err"
rc=$?; echo "exr: $(cut -c1-160 $O/bench_exr.json)"; stop $rc
timeout -k 10 600 python3 bench.py --workload c4 --steps 10 --warmup 2 > "$O/bench_c4.json" 2> "$O/bench_c4.err"
rc=$?; echo "c4: $(cut -c1-160 $O/bench_c4.json)"; stop $rc
