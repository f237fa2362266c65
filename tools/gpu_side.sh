#!/bin/bash
# GPU box: the non-default workloads (C2, C3+DRI, C4 encode, C5 PNG, HDR read) with their CPU
# baselines and parity checks, plus rocprofv3 kernel stats of C4 and C5. Outputs under
# gpurun_out/side (copied into profiles/ after).
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/side"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for w in ${SIDE_WORKLOADS:-c2 c3dri c4 c5 hdr hdrflat}; do
  timeout -k 10 300 python3 "$R/bench.py" --workload $w --steps 3 > "$O/bench_$w.json" 2> "$O/bench_$w.err"
  echo "$w: $(cut -c1-160 $O/bench_$w.json)"
done
for w in ${SIDE_PROF:-c4 c5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$w" -o run -- python3 "$R/bench.py" --workload $w --steps 2 --no-cpu > "$O/rocprof_$w.json" 2> "$O/rocprof_$w.err"
  echo "rocprof $w done"
done
