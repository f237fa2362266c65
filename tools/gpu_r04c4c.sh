#!/bin/bash
# Round 4: k_enc_units time, old vs dword-gather build (rocprofv3 kernel stats, C4 bench).
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
O="$R/gpurun_out/r04c4c"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in encold new; do
  if [ $v = new ]; then unset ICX_LIB; else export ICX_LIB=$R/imagecodecs_amd/exp/libicx_encold.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$v" -o run -- python3 "$R/bench.py" --workload c4 --steps 10 --warmup 2 --no-cpu > "$O/$v.json" 2> "$O/$v.err"
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -E "k_enc_units|k_enc_emit" "$O/$v/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-40,100-200
done
