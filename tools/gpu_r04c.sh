#!/bin/bash
# Round 4 measurements: C2 kernel trace (both entropy paths), C3 with staggered pipelines.
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/${TAG:-r04c}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for gw in 0 1; do
  ICX_GW=$gw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c2_gw$gw" -o run -- \
    python3 "$R/bench.py" --workload c2 --steps 5 --warmup 1 --no-cpu --no-pcie > "$O/c2_gw$gw.json" 2> "$O/c2_gw$gw.err"
  echo "c2 gw=$gw: $(python3 -c "import json;d=json.load(open('$O/c2_gw$gw.json'));print(d['value'],d['ms_per_step'])")"
done
for v in "" "ICX_STAGGER=1" "" "ICX_STAGGER=1"; do
  env $v timeout -k 10 300 python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu --no-pcie > "$O/c3.json" 2> "$O/c3.err"
  echo "c3 ${v:-default}: $(python3 -c "import json;d=json.load(open('$O/c3.json'));print(d['value'],d['ms_per_step'])")"
done
