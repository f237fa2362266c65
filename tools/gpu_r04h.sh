#!/bin/bash
# Round 4: graph capture with explicit event-record nodes (probe), then C2 / C3 in graph mode and
# without, then the GPU suite.
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd "$R"; mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 5 60 ./tools/graph_ev2; rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
for e in "c2:" "c2:ICX_GRAPH=0" "c3:" "c3:ICX_GRAPH=0" "c2:" "c2:ICX_GRAPH=0" "c3:" "c3:ICX_GRAPH=0"; do
  w=${e%%:*}; v=${e#*:}
  env $v timeout -k 10 200 python3 bench.py --workload $w --no-cpu --no-pcie --steps 10 --warmup 2 > gpurun_out/r04h_ab.json 2>gpurun_out/r04h_ab.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04h_ab.err; stop $rc; exit 1; }
  echo "$w ${v:-graph}: $(python3 -c "import json;d=json.load(open('gpurun_out/r04h_ab.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['stage_ms'])")"
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04h_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04h_tests.log)"; stop $rc
grep -E "^FAILED|^ERROR|GPU IDAT" gpurun_out/r04h_tests.log | head -20
