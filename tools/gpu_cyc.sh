#!/bin/bash
# Write-pass cycle study (timing experiments only): for each experiment library named in LIBS
# (built with -DICX_EXP_CYC), one ICX_PIPES=1 bench step; prints the mean of the sampled waves'
# cycles per loop iteration. Output under gpurun_out/cyc_<lib>.log.
set -e
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
for L in $LIBS; do
    ICX_PIPES=1 ICX_LIB="$R/imagecodecs_amd/exp/libicx_$L.so" timeout -k 10 200 python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-pcie > "$R/gpurun_out/cyc_$L.log" 2>&1
    python3 - "$R/gpurun_out/cyc_$L.log" "$L" <<'PY'
import sys, re
v = [int(m.group(1)) for m in re.finditer(r"per_iter (\d+)", open(sys.argv[1]).read())]
it = [int(m.group(1)) for m in re.finditer(r"iters (\d+)", open(sys.argv[1]).read())]
print(f"{sys.argv[2]:10s} waves {len(v)} mean cycles/iter {sum(v)/max(1,len(v)):.0f} min {min(v) if v else 0} max {max(v) if v else 0} iters {sum(it)/max(1,len(it)):.0f}")
PY
done
