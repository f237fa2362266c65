#!/bin/bash
# Round 4: GPU suite on the committed tree; k_gw_lane fetch vs guess lead (PMC); C2 at the
# driver's settings with its kernel trace.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04k_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04k_tests.log)"; stop $rc
grep -E "^FAILED|^ERROR" gpurun_out/r04k_tests.log | head -15
for lead in 4096 2048 1024 256; do
  ICX_GUESS_LEAD=$lead timeout -k 10 400 python3 tools/pmc_traffic.py run --workload c3 --images 128 --kernel k_gw_lane --out gpurun_out/r04k_lead$lead.json > gpurun_out/r04k_lead$lead.log 2>&1
  rc=$?; stop $rc
  echo "lead $lead: $(python3 -c "import json;d=json.load(open('gpurun_out/r04k_lead$lead.json'));print(d['fetch_bytes']/1e6/d['images_per_launch'], d['write_bytes']/1e6/d['images_per_launch'], d['images_per_launch'])" 2>&1)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04k_c2" -o run -- python3 "$R/bench.py" --workload c2 --steps 20 --warmup 5 > "$R/gpurun_out/r04k_c2_rocprof.json" 2> "$R/gpurun_out/r04k_c2_rocprof.err"
rc=$?; stop $rc
cd "$R"
timeout -k 10 400 python3 bench.py --workload c2 --steps 20 --warmup 5 > gpurun_out/r04k_bench_c2.json 2> gpurun_out/r04k_bench_c2.err
rc=$?; stop $rc
python3 -c "import json;d=json.load(open('gpurun_out/r04k_bench_c2.json'));print('c2',d['value'],d['ms_per_step'],d['entropy_paths'],d['parity'])"
