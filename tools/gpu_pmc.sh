#!/bin/bash
# PMC passes on the GPU box, one rocprofv3 --pmc run per pass (no tracing domains), over a short
# bench (default: one C3 group of 128 images, one pipeline, so each kernel runs alone).
#   LABEL=r05p PASSES="SQ_WAVES SQ_WAVE_CYCLES;SQ_INSTS_LDS GRBM_GUI_ACTIVE" tools/gpu_pmc.sh
# Env: LIB (library under imagecodecs_amd/, default lib/libicx.so), BENCH_ARGS, PIPES (default 1),
# LIST=1 also writes `rocprofv3 -L` to gpurun_out/<LABEL>_counters.txt.
# Output: gpurun_out/<LABEL>_pmc<k>/ (CSV) and gpurun_out/<LABEL>_sq.txt (tools/sq_summary.py).
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R=$(pwd)
cd /tmp && export TMPDIR=/tmp
L="${LABEL:-pmc}"
mkdir -p "$R/gpurun_out"
if [ -n "${LIST:-}" ]; then
  timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/${L}_counters.txt" 2>&1 || echo "counter list rc=$?"
fi
k=0
dirs=""
IFS=';' read -ra PS <<< "${PASSES:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY}"
for p in "${PS[@]}"; do
  k=$((k + 1))
  d="$R/gpurun_out/${L}_pmc$k"
  ICX_PIPES="${PIPES:-1}" ICX_LIB="$R/imagecodecs_amd/${LIB:-lib/libicx.so}" timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$d" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --no-pcie ${BENCH_ARGS:---images 128} > "$d.log" 2>&1
  rc=$?
  echo "pass $k ($p) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$d.log"; exit $rc; }
  dirs="$dirs $d"
done
python3 "$R/tools/sq_summary.py" $dirs > "$R/gpurun_out/${L}_sq.txt" 2>&1
head -30 "$R/gpurun_out/${L}_sq.txt"
